"""Synthetic Kaldi-style inputs for the feature front-end tests (apply-cmvn / add-deltas):
utterances of several speakers (including 1- and 2-frame ones and ones longer than
max_seq_length), per-speaker double-precision CMVN statistics, an utt2spk table, one utterance
whose speaker has no statistics and one without labels."""
import os
import struct

import numpy as np


def make(seed=0, n_utt=18, D=13):
    rs = np.random.RandomState(seed)
    fea, u2s, lab = {}, {}, {}
    lens = [1, 2, 3, 5] + list(rs.randint(20, 160, n_utt - 4))
    for i, T in enumerate(lens):
        spk = "spk%d" % (i % 4)
        k = "%s_u%03d" % (spk, i)
        fea[k] = (rs.randn(T, D) * rs.uniform(0.5, 4) + rs.randn(1, D) * 3).astype(np.float32)
        u2s[k] = spk
        lab[k] = rs.randint(3, 50, T).astype(np.int32)
    # speaker statistics over that speaker's frames, as compute-cmvn-stats accumulates them
    stats = {}
    for spk in sorted(set(u2s.values())):
        x = np.concatenate([fea[k] for k in fea if u2s[k] == spk]).astype(np.float64)
        s = np.zeros((2, D + 1))
        s[0, :D], s[1, :D], s[0, D] = x.sum(0), (x * x).sum(0), len(x)
        stats[spk] = s
    # a speaker without statistics (apply-cmvn drops its utterances) and an utterance without labels
    fea["spkX_u999"] = rs.randn(40, D).astype(np.float32)
    u2s["spkX_u999"] = "spkX"
    lab["spkX_u999"] = rs.randint(3, 50, 40).astype(np.int32)
    fea["spk1_nolab"] = rs.randn(33, D).astype(np.float32)
    u2s["spk1_nolab"] = "spk1"
    return fea, u2s, stats, lab


def dm_bytes(key, m):
    m = np.ascontiguousarray(m, dtype="<f8")
    return ((key + " ").encode() + b"\0BDM \x04" + struct.pack("<i", m.shape[0]) + b"\x04" +
            struct.pack("<i", m.shape[1]) + m.tobytes())


def write_files(d, stats, u2s, text_stats=False):
    cm, us = os.path.join(d, "cmvn.ark"), os.path.join(d, "utt2spk")
    with open(cm, "wb") as f:
        for k, m in stats.items():
            if text_stats:
                f.write(("%s  [\n" % k).encode())
                for r in m:
                    f.write((" ".join(repr(float(v)) for v in r) + "\n").encode())
                f.write(b" ]\n")
            else:
                f.write(dm_bytes(k, m))
    with open(us, "w") as f:
        for k, s in u2s.items():
            f.write("%s %s\n" % (k, s))
    return cm, us


def fea_opts(cm, us, order=2, norm_vars=None):
    nv = "" if norm_vars is None else " --norm-vars=%s" % ("true" if norm_vars else "false")
    return ("apply-cmvn --utt2spk=ark:%s%s  ark:%s ark:- ark:- | add-deltas --delta-order=%d "
            "ark:- ark:- |" % (us, nv, cm, order))
