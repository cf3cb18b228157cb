"""pkc.data_io — Kaldi ark I/O and chunk preparation for the pkc run_nn.

Host side (parsing, utterance bookkeeping) mirrors data_io.py:16-88 (load_dataset) and the
kaldi-io readers; the numeric chunk preparation of data_io.py:105-145 (context window, chunk
z-normalisation) and the frame shuffle of data_io.py:269-270 run on the GPU (pkc_cw_stats /
pkc_cw_apply) so only raw 40-dim frames cross PCIe.
"""
import ctypes as C
import struct

import numpy as np
import torch

from . import _lib as L
from ._lib import call, ptr


# ------------------------------------------------------------------------------------------ ark I/O
def write_mat_path(path, m, key="", append=False):
    """data_io.write_mat byte layout (data_io.py:770-806), via the C ABI (pkc_ark_write_mat)."""
    m = np.ascontiguousarray(m, dtype=np.float32)
    call("pkc_ark_write_mat", path.encode(), int(append), key.encode(), m.shape[0], m.shape[1],
         m.ctypes.data_as(C.c_void_p))


def read_mat_ark_path(path):
    """Binary FM/DM/CM ark -> generator of (key, float32 matrix) (data_io.py:645-766)."""
    lib = L.lib()
    n = lib.pkc_ark_index(path.encode(), None, None, None, 0, None, 0)
    if n == L.PKC_ERR_UNSUPPORTED:         # compressed matrices: parse the bytes (pkc_ark_decode_cm)
        with open(path, "rb") as f:
            yield from parse_mat_ark_bytes(f.read())
        return
    if n < 0:
        raise L.PkcError(lib.pkc_last_error().decode())
    offs, rows, cols = (C.c_int64 * n)(), (C.c_int64 * n)(), (C.c_int64 * n)()
    kcap = 1 << 20
    kbuf = C.create_string_buffer(kcap)
    lib.pkc_ark_index(path.encode(), offs, rows, cols, n, kbuf, kcap)
    keys = kbuf.raw.split(b"\0")[:n]
    for i in range(n):
        c = abs(cols[i])
        out = np.empty((rows[i], c), dtype=np.float32)
        call("pkc_ark_read_rows", path.encode(), offs[i], rows[i], cols[i],
             out.ctypes.data_as(C.c_void_p))
        yield keys[i].decode("latin1"), out


def parse_mat_ark_bytes(buf):
    """Binary FM/DM ark held in memory (e.g. a Kaldi pipe's stdout) -> [(key, float32 matrix)]."""
    out, pos = [], 0
    while pos < len(buf):
        sp = buf.index(b" ", pos)
        key = buf[pos:sp].decode("latin1").strip()
        pos = sp + 1
        if buf[pos:pos + 2] != b"\0B":
            raise ValueError("only binary matrices are supported")
        hdr = buf[pos + 2:pos + 5]
        if hdr == b"CM ":
            out.append((key, decode_cm(buf, pos + 5)))
            pos += 5 + int(L.lib().pkc_ark_cm_size(_addr(buf, pos + 5), len(buf) - pos - 5))
            continue
        dt = {b"FM ": np.float32, b"DM ": np.float64}.get(hdr)
        if dt is None:
            raise ValueError("unsupported matrix type %r (CM2 / CM3 are not supported, as in "
                             "data_io.py:736)" % hdr)
        rows = struct.unpack("<i", buf[pos + 6:pos + 10])[0]
        cols = struct.unpack("<i", buf[pos + 11:pos + 15])[0]
        pos += 15
        n = rows * cols * np.dtype(dt).itemsize
        out.append((key, np.frombuffer(buf[pos:pos + n], dtype=dt).reshape(rows, cols)
                    .astype(np.float32)))
        pos += n
    return out


def _addr(buf, off):
    a = np.frombuffer(buf, dtype=np.uint8)
    return C.c_void_p(a.ctypes.data + off)


def decode_cm(buf, off):
    """One "CM " compressed matrix whose global header starts at buf[off] -> float32 matrix."""
    lib = L.lib()
    n = len(buf) - off
    size = lib.pkc_ark_cm_size(_addr(buf, off), n)
    if size < 0 or size > n:
        raise ValueError("truncated compressed matrix")
    rows, cols = struct.unpack("<ii", buf[off + 8:off + 16])
    out = np.empty((rows, cols), dtype=np.float32)
    call("pkc_ark_decode_cm", _addr(buf, off), n, out.ctypes.data_as(C.c_void_p))
    return out


def read_vec_int_ark_path(path):
    """Binary int32-vector ark (alignments after ali-to-pdf) -> generator (data_io.py:412-455)."""
    with open(path, "rb") as f:
        buf = f.read()
    return parse_vec_int_ark_bytes(buf)


def parse_vec_int_ark_bytes(buf):
    pos = 0
    while pos < len(buf):
        sp = buf.index(b" ", pos)
        key = buf[pos:sp].decode("latin1").strip()
        pos = sp + 1
        if buf[pos:pos + 2] != b"\0B":
            raise ValueError("only binary int vectors are supported")
        n = struct.unpack("<i", buf[pos + 3:pos + 7])[0]
        pos += 7
        rec = np.frombuffer(buf[pos:pos + 5 * n], dtype=[("size", "i1"), ("value", "<i4")])
        pos += 5 * n
        yield key, rec["value"].astype(np.int32)


def write_vec_int_path(path, v, key, append=False):
    v = np.asarray(v, dtype=np.int32)
    rec = np.empty(len(v), dtype=[("size", "i1"), ("value", "<i4")])
    rec["size"] = 4
    rec["value"] = v
    with open(path, "ab" if append else "wb") as f:
        f.write((key + " ").encode("latin1") + b"\0B\x04" + struct.pack("<i", len(v)) + rec.tobytes())


def load_counts(path):
    """data_io.py:148-152."""
    with open(path) as f:
        row = next(f).strip().strip("[]").strip()
    return np.array([np.float32(v) for v in row.split()])


# --------------------------------------------------------------------------------- chunk assembly
def load_dataset(fea, labs, max_sequence_length):
    """Utterance bookkeeping of data_io.py:16-88 on in-memory dicts.

    fea: {key: (T, D) float32}; labs: list of {key: (T,) int} (one per label stream) or [].
    Returns names, raw (N, D) float32, [label arrays (N,)], end_index."""
    if labs:
        keep = set(fea)
        for l in labs:
            keep &= set(l)
        fea = {k: v for k, v in fea.items() if k in keep}
    names, fc, lc = [], [], [[] for _ in labs]
    for k in sorted(sorted(fea), key=lambda k: len(fea[k])):
        f = fea[k]
        T = len(f)
        m = max_sequence_length
        if m > 0 and T > m:
            start, j = 0, 0
            while True:
                if T - start > m + m / 4:
                    stop = start + m
                else:
                    stop = T
                fc.append(f[start:stop])
                for li, l in enumerate(labs):
                    lc[li].append(l[k][start:stop])
                names.append("%s_split%d" % (k, j))
                if stop == T:
                    break
                start, j = stop, j + 1
        else:
            fc.append(f)
            for li, l in enumerate(labs):
                lc[li].append(l[k])
            names.append(k)
    order = sorted(range(len(fc)), key=lambda i: fc[i].shape[0])
    fc = [fc[i] for i in order]
    names = [names[i] for i in order]
    lab_arrays = [np.concatenate([l[i] for i in order]) for l in lc]
    end_index = np.cumsum([x.shape[0] for x in fc])
    return names, np.concatenate(fc).astype(np.float32), lab_arrays, end_index


class Chunk:
    """A prepared chunk resident in HBM: feats (Nout, C) fp32, labels (Nout, nlab) int32."""

    def __init__(self, names, end_index, feats, labels, fea_cols, lab_names):
        self.names, self.end_index = names, end_index
        self.feats, self.labels = feats, labels
        self.fea_cols, self.lab_names = fea_cols, lab_names

    @property
    def n_rows(self):
        return self.feats.shape[0]


class StagedChunk:
    """A chunk after the host half of loading: utterances sorted / split (load_dataset) and the
    raw frames on their way to HBM — copied from pinned host memory by an asynchronous copy on a
    dedicated stream (hipMemcpyAsync underneath), so the upload of chunk k+1 overlaps the
    training of chunk k (run_nn stages the next chunk from its loader thread)."""

    def __init__(self, names, raw, lab_arrays, end_index, device):
        self.names, self.lab_arrays, self.end_index = names, lab_arrays, end_index
        self.shape = raw.shape
        dev = torch.device(device)
        self.stream = torch.cuda.Stream(device=dev)
        pinned = torch.empty(raw.shape, dtype=torch.float32, pin_memory=True)
        pinned.numpy()[...] = raw
        with torch.cuda.stream(self.stream):
            self.raw_d = pinned.to(dev, non_blocking=True)
            self.done = torch.cuda.Event()
            self.done.record(self.stream)
        self._pinned = pinned           # alive until the copy has completed (finish_chunk)


def stage_chunk(fea, labs, max_sequence_length, device="cuda"):
    names, raw, lab_arrays, end_index = load_dataset(fea, labs, max_sequence_length)
    return StagedChunk(names, np.ascontiguousarray(raw, dtype=np.float32), lab_arrays, end_index,
                       device)


def prepare_chunk(fea, labs, lab_names, left, right, max_sequence_length, shuffle_rng=None,
                  device="cuda", fea_name="fea", staged=None):
    """data_io.load_chunk + read_lab_fea for one feature stream (data_io.py:121-145, 155-282):
    context window, chunk z-normalisation, label shift by the chunk minimum, optional frame
    shuffle (rng: the RandomState the reference's global np.random would be, seeded by run_nn).
    staged: the StagedChunk of these utterances when the loader thread already uploaded them."""
    if staged is None:
        staged = stage_chunk(fea, labs, max_sequence_length, device)
    names, lab_arrays, end_index = staged.names, staged.lab_arrays, staged.end_index
    N, D = staged.shape
    Nout = N - left - right
    end_index = end_index - left
    end_index[-1] = end_index[-1] - right
    Cc = D * (left + right + 1)
    lab_cols = []
    for la in lab_arrays:                      # data_io.py:137-141
        la = la - la.min()
        lab_cols.append(la[left:N - right] if right > 0 else la[left:])
    labels = np.stack(lab_cols, 1).astype(np.int32) if lab_cols else np.zeros((Nout, 0), np.int32)
    perm = None
    if shuffle_rng is not None:                # same draws as shuffling the (Nout, C) matrix rows
        perm = np.arange(Nout, dtype=np.int64)
        shuffle_rng.shuffle(perm)
        labels = labels[perm]
    dev = torch.device(device)
    torch.cuda.current_stream(dev).wait_event(staged.done)
    raw_d = staged.raw_d
    raw_d.record_stream(torch.cuda.current_stream(dev))
    mean = torch.empty(Cc, dtype=torch.float64, device=dev)
    std = torch.empty(Cc, dtype=torch.float64, device=dev)
    work = torch.empty(int(L.lib().pkc_cw_stats_work_size(N, D, left, right)), dtype=torch.float64,
                       device=dev)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    call("pkc_cw_stats", ptr(raw_d), N, D, left, right, ptr(mean), ptr(std), ptr(work), s)
    feats = torch.empty(Nout, Cc, dtype=torch.float32, device=dev)
    perm_d = torch.from_numpy(perm).to(dev) if perm is not None else None
    call("pkc_cw_apply", ptr(raw_d), N, D, left, right, ptr(mean), ptr(std), ptr(perm_d), ptr(feats),
         Cc, s)
    labels_d = torch.from_numpy(np.ascontiguousarray(labels)).to(dev)
    return Chunk(names, end_index, feats, labels_d, {fea_name: (0, Cc)}, list(lab_names))
