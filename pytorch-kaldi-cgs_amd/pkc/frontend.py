"""pkc.frontend — the Kaldi feature front-end of the reference's feature pipe, without Kaldi.

The reference reads every feature stream through a shell pipe (data_io.py:18, read_mat_ark
data_io.py:645-664)::

    copy-feats scp:<fea_lst> ark:- |apply-cmvn --utt2spk=ark:<utt2spk> ark:<cmvn.ark> ark:- ark:- |
        add-deltas --delta-order=<N> ark:- ark:- |

(the fea_opts of every shipped cfg).  ``FeaFrontend.parse`` recognises that pipe; the host does
the once-per-chunk bookkeeping Kaldi does per speaker (the ApplyCmvn offsets / scales, the
DeltaFeatures windows, both in Kaldi's own float / double arithmetic) and ``pkc_feat_frontend``
applies them to every frame on the GPU (pytorch-kaldi-cgs_amd/csrc/pkc_frontend.hip).

Kaldi itself is a third-party dependency that is not in /root/reference (no binaries, no fixture
of its output), so this restatement is parity-UNPINNED against Kaldi; it is checked bit-exactly
against the independent C restatement in oracle/kaldi_feat.c.
"""
import os
import re
import shlex
import struct

import numpy as np


def _strtobool(v):
    return str(v).strip().lower() in ("true", "1", "yes", "t")


def _rspec_path(spec, what):
    if not spec.startswith("ark:"):
        raise NotImplementedError("%s: only ark: rspecifiers are read natively (got %r)" % (what, spec))
    path = spec[4:]
    for opt in ("s,", "cs,", "o,", "p,", "t,", "b,"):   # ark,s,cs:... style flags
        if path.startswith(opt):
            path = path[len(opt):]
    return path


def read_utt2spk(path):
    """Kaldi text table ``utt spk`` (one pair per line)."""
    m = {}
    with open(path) as f:
        for line in f:
            p = line.split()
            if len(p) >= 2:
                m[p[0]] = p[1]
    return m


def parse_stats_ark(buf):
    """CMVN statistics archive: binary (``\\0BDM ``/``\\0BFM ``) or text (``key [ ... ]``) matrices
    -> {key: float64 (rows, cols)} (the double precision ApplyCmvn reads them in)."""
    out, pos = {}, 0
    n = len(buf)
    while pos < n:
        while pos < n and buf[pos:pos + 1].isspace():
            pos += 1
        if pos >= n:
            break
        sp = buf.index(b" ", pos)
        key = buf[pos:sp].decode("latin1")
        pos = sp + 1
        if buf[pos:pos + 2] == b"\0B":
            hdr = buf[pos + 2:pos + 5]
            dt = {b"DM ": "<f8", b"FM ": "<f4"}.get(hdr)
            if dt is None:
                raise ValueError("cmvn stats: unsupported matrix type %r" % hdr)
            rows = struct.unpack("<i", buf[pos + 6:pos + 10])[0]
            cols = struct.unpack("<i", buf[pos + 11:pos + 15])[0]
            pos += 15
            nb = rows * cols * np.dtype(dt).itemsize
            out[key] = np.frombuffer(buf[pos:pos + nb], dtype=dt).reshape(rows, cols).astype(np.float64)
            pos += nb
        else:
            end = buf.index(b"]", pos)
            body = buf[pos:end].decode("latin1").replace("[", " ").strip()
            rows = [list(map(float, r.split())) for r in body.split("\n") if r.strip()]
            out[key] = np.array(rows, dtype=np.float64)
            pos = end + 1
    return out


def cmvn_norm(stats, norm_vars):
    """transform/cmvn.cc ApplyCmvn: per-dimension float (offset, scale) of one stats matrix.

    means only: offset = (float)((double)(float)(-1/count) * sum)   (Vector<float>::AddVec with a
    float alpha over a double vector); means+vars: mean, var = sum/count, sumsq/count - mean^2
    (floored at 1e-20), scale = 1/sqrt(var), offset = -(mean*scale), both stored as float."""
    stats = np.asarray(stats, dtype=np.float64)
    dim = stats.shape[1] - 1
    count = float(stats[0, dim])
    if count < 1.0:
        raise ValueError("Insufficient stats for cepstral mean and variance normalization: "
                         "count = %g" % count)
    if not norm_vars:
        alpha = float(np.float32(-1.0 / count))
        offset = (alpha * stats[0, :dim]).astype(np.float32)
        return offset, np.ones(dim, np.float32)
    if stats.shape[0] < 2:
        raise ValueError("apply-cmvn --norm-vars=true needs 2-row stats")
    mean = stats[0, :dim] / count
    var = stats[1, :dim] / count - mean * mean
    var = np.where(var < 1.0e-20, 1.0e-20, var)
    scale = 1.0 / np.sqrt(var)
    if not np.all(np.isfinite(scale)) or np.any(1.0 / scale == 0.0):
        raise ValueError("NaN or infinity in cepstral mean/variance computation")
    offset = -(mean * scale)
    return offset.astype(np.float32), scale.astype(np.float32)


def delta_scales(order, window):
    """feat/feature-functions.cc DeltaFeatures::DeltaFeatures in float arithmetic: scales[0] = [1];
    scales[i] = (scales[i-1] convolved with j = -window..window) * (float)(1/sum j^2).
    Returns (order+1, 2*maxoff+1) float32 with each order's window centred, zero elsewhere."""
    if not (0 <= order < 1000 and 0 < window < 1000):
        raise ValueError("add-deltas: bad order/window")
    f32 = np.float32
    scales = [np.array([1.0], f32)]
    for i in range(1, order + 1):
        prev = scales[-1]
        po = (len(prev) - 1) // 2
        co = po + window
        cur = np.zeros(len(prev) + 2 * window, f32)
        normalizer = f32(0.0)
        for j in range(-window, window + 1):
            normalizer = f32(normalizer + f32(j * j))
            for k in range(-po, po + 1):
                cur[j + k + co] = f32(cur[j + k + co] + f32(f32(j) * prev[k + po]))
        alpha = f32(1.0 / float(normalizer))
        cur = (cur * alpha).astype(f32)
        scales.append(cur)
    maxoff = order * window
    tab = np.zeros((order + 1, 2 * maxoff + 1), f32)
    for i, sc in enumerate(scales):
        o = (len(sc) - 1) // 2
        tab[i, maxoff - o:maxoff + o + 1] = sc
    return tab, maxoff


class FeaFrontend:
    """apply-cmvn / add-deltas stages of one fea_opts pipe."""

    def __init__(self):
        self.cmvn = None          # dict(stats={key: (2, D+1) f64}, utt2spk={utt: spk} | None, vars)
        self.order, self.window = 0, 2

    @staticmethod
    def parse(fea_opts):
        """fea_opts -> FeaFrontend (None for an empty pipe).  Stages other than apply-cmvn and
        add-deltas (and options Kaldi does not have) raise NotImplementedError."""
        fe = FeaFrontend()
        stages = [s.strip() for s in fea_opts.split("|") if s.strip()]
        if not stages:
            return None
        for st in stages:
            argv = shlex.split(st)
            prog, args = argv[0], argv[1:]
            opts = [a for a in args if a.startswith("--")]
            pos = [a for a in args if not a.startswith("--")]
            kv = {}
            for o in opts:
                k, _, v = o[2:].partition("=")
                kv[k.replace("_", "-")] = v
            if prog == "apply-cmvn":
                if fe.cmvn is not None or fe.order:
                    raise NotImplementedError("fea_opts: apply-cmvn after add-deltas / twice")
                unknown = set(kv) - {"utt2spk", "norm-vars", "norm-means", "reverse"}
                if unknown or _strtobool(kv.get("reverse", "false")):
                    raise NotImplementedError("apply-cmvn options %s" % sorted(kv))
                if len(pos) != 3 or pos[1:] != ["ark:-", "ark:-"]:
                    raise NotImplementedError("apply-cmvn %s: expected <cmvn-rspecifier> ark:- ark:-"
                                              % " ".join(pos))
                norm_means = _strtobool(kv.get("norm-means", "true"))
                norm_vars = _strtobool(kv.get("norm-vars", "false"))
                if norm_vars and not norm_means:
                    raise ValueError("You cannot normalize the variance but not the mean.")
                u2s = kv.get("utt2spk")
                with open(_rspec_path(pos[0], "apply-cmvn stats"), "rb") as f:
                    stats = parse_stats_ark(f.read())
                fe.cmvn = dict(stats=stats, utt2spk=read_utt2spk(_rspec_path(u2s, "utt2spk"))
                               if u2s else None, norm_vars=norm_vars, norm_means=norm_means)
            elif prog == "add-deltas":
                unknown = set(kv) - {"delta-order", "delta-window"}
                if unknown:
                    raise NotImplementedError("add-deltas options %s" % sorted(kv))
                if pos != ["ark:-", "ark:-"]:
                    raise NotImplementedError("add-deltas %s" % " ".join(pos))
                fe.order = int(kv.get("delta-order", "2"))
                fe.window = int(kv.get("delta-window", "2"))
                if fe.order > 7:
                    raise NotImplementedError("add-deltas --delta-order > 7")
            else:
                raise NotImplementedError("fea_opts stage %r has no native pkc implementation" % prog)
        return fe

    def out_dim(self, D):
        return D * (self.order + 1)

    def norm_tables(self, keys, D):
        """(kept keys, norm (n, 2, D) float32 {offset, scale}, norm index per kept key, cmvn_mode).
        Utterances without statistics are dropped, as apply-cmvn drops them (it warns and writes
        nothing for them)."""
        if self.cmvn is None or not self.cmvn["norm_means"]:
            return list(keys), np.zeros((0, 2, D), np.float32), np.zeros(len(keys), np.int32), 0
        stats, u2s = self.cmvn["stats"], self.cmvn["utt2spk"]
        kept, idx, spk_index, tabs = [], [], {}, []
        for k in keys:
            sk = u2s.get(k) if u2s is not None else k
            if sk is None or sk not in stats:
                continue
            if sk not in spk_index:
                st = stats[sk]
                if st.shape[1] - 1 != D:
                    raise ValueError("cmvn stats dimension %d != feature dimension %d"
                                     % (st.shape[1] - 1, D))
                off, sc = cmvn_norm(st, self.cmvn["norm_vars"])
                spk_index[sk] = len(tabs)
                tabs.append(np.stack([off, sc]))
            kept.append(k)
            idx.append(spk_index[sk])
        norm = np.stack(tabs).astype(np.float32) if tabs else np.zeros((0, 2, D), np.float32)
        return kept, norm, np.asarray(idx, np.int32), 2 if self.cmvn["norm_vars"] else 1


def kaldi_on_path():
    return any(os.access(os.path.join(d, "copy-feats"), os.X_OK)
               for d in os.environ.get("PATH", "").split(os.pathsep) if d)


_PIPE_RE = re.compile(r"^\s*(apply-cmvn|add-deltas)\b")


def is_native_pipe(fea_opts):
    """True when every stage of fea_opts is one pkc runs itself."""
    stages = [s for s in fea_opts.split("|") if s.strip()]
    return bool(stages) and all(_PIPE_RE.match(s) for s in stages)
