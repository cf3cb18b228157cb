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
    """Binary FM/DM/CM or text ark -> generator of (key, float32 matrix) (data_io.py:645-766)."""
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


def _readline(buf, pos):
    """The bytes of buf from pos through the next newline (file.readline), and the new position."""
    nl = buf.find(b"\n", pos)
    end = len(buf) if nl < 0 else nl + 1
    return buf[pos:end], end


def _read_mat_ascii(buf, pos):
    """Text matrix body after its " [" (data_io.py:714-726, reached from read_mat :680-681): the
    rest of the "[" line is skipped, then one row per line until a line whose last token is "]";
    tokens parsed as float32 (numpy's str -> float32, as there).  Returns (matrix, new pos)."""
    _, pos = _readline(buf, pos)
    rows = []
    while True:
        line, pos = _readline(buf, pos)
        if not line:
            raise ValueError("text matrix ends before its ']'")
        arr = line.decode().strip().split()
        if not arr:
            continue
        if arr[-1] != "]":
            rows.append(np.array(arr, dtype=np.float32))
        else:
            rows.append(np.array(arr[:-1], dtype=np.float32))
            return np.vstack(rows), pos


def parse_mat_ark_bytes(buf):
    """FM / DM / CM binary or text (`ark,t:`) matrix ark held in memory (e.g. a Kaldi pipe's
    stdout) -> [(key, float32 matrix)]; text and binary entries may alternate (read_mat decides per
    entry, data_io.py:669-684)."""
    out, pos = [], 0
    while pos < len(buf):
        if not buf[pos:].strip():            # read_key: an empty key ends the ark (:399)
            break
        sp = buf.index(b" ", pos)
        key = buf[pos:sp].decode("latin1").strip()
        pos = sp + 1
        if buf[pos:pos + 2] == b" [":
            m, pos = _read_mat_ascii(buf, pos + 2)
            out.append((key, m))
            continue
        if buf[pos:pos + 2] != b"\0B":
            raise ValueError("%s: neither a binary matrix nor a text one (' [')" % key)
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
    """Binary or text int32-vector ark (alignments after ali-to-pdf) -> generator
    (data_io.py:412-455)."""
    with open(path, "rb") as f:
        buf = f.read()
    return parse_vec_int_ark_bytes(buf)


def parse_vec_int_ark_bytes(buf):
    """Binary or text int-vector ark -> generator of (key, int32 vector) (read_vec_int,
    data_io.py:431-455: the text form is the rest of the line, optional "[" / "]" tokens removed)."""
    pos = 0
    while pos < len(buf):
        if not buf[pos:].strip():
            break
        sp = buf.index(b" ", pos)
        key = buf[pos:sp].decode("latin1").strip()
        pos = sp + 1
        if buf[pos:pos + 2] != b"\0B":
            line, pos = _readline(buf, pos)
            arr = line.decode().strip().split()
            try:                              # :448-452 (a missing "[" leaves a "]" in place)
                arr.remove("[")
                arr.remove("]")
            except ValueError:
                pass
            yield key, np.array(arr, dtype=np.int64).astype(np.int32)
            continue
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
def dataset_pieces(lengths, labs, max_sequence_length):
    """Utterance bookkeeping of data_io.py:16-88 on lengths only.

    lengths: {key: T}; labs: list of {key: (T,) int} (one per label stream) or [].
    Returns names (first-sort order, as the reference returns snt_name), pieces [(key, start,
    stop)] in the final (length-sorted) order, [label arrays (N,)], end_index."""
    if labs:
        keep = set(lengths)
        for l in labs:
            keep &= set(l)
        lengths = {k: v for k, v in lengths.items() if k in keep}
    names, pieces = [], []
    for k in sorted(sorted(lengths), key=lambda k: lengths[k]):       # data_io.py:34
        T = lengths[k]
        m = max_sequence_length
        if m > 0 and T > m:                                            # data_io.py:41-60
            start, j = 0, 0
            while True:
                if T - start > m + m / 4:
                    stop = start + m
                else:
                    stop = T
                pieces.append((k, start, stop))
                names.append("%s_split%d" % (k, j))
                if stop == T:
                    break
                start, j = stop, j + 1
        else:
            pieces.append((k, 0, T))
            names.append(k)
    # :77-79 re-sorts the pieces by length (stable) but NOT snt_name, which keeps the order of
    # the first sort (visible once pieces were split; forward mode never splits, data_io.py:176)
    order = sorted(range(len(pieces)), key=lambda i: pieces[i][2] - pieces[i][1])
    pieces = [pieces[i] for i in order]
    lab_arrays = [np.concatenate([l[k][a:b] for k, a, b in pieces]) for l in labs]
    end_index = np.cumsum([b - a for _, a, b in pieces])
    return names, pieces, lab_arrays, end_index


def load_dataset(fea, labs, max_sequence_length):
    """data_io.py:16-88 on in-memory dicts.

    fea: {key: (T, D) float32}; labs: list of {key: (T,) int} (one per label stream) or [].
    Returns names, raw (N, D) float32, [label arrays (N,)], end_index."""
    names, pieces, lab_arrays, end_index = dataset_pieces({k: len(v) for k, v in fea.items()},
                                                          labs, max_sequence_length)
    raw = np.concatenate([fea[k][a:b] for k, a, b in pieces]).astype(np.float32)
    return names, raw, lab_arrays, end_index


class Chunk:
    """A prepared chunk resident in HBM: feats (Nout, C) fp32, labels (Nout, nlab) int32."""

    def __init__(self, names, end_index, feats, labels, fea_cols, lab_names):
        self.names, self.end_index = names, end_index
        self.feats, self.labels = feats, labels
        self.fea_cols, self.lab_names = fea_cols, lab_names

    @property
    def n_rows(self):
        return self.feats.shape[0]

    @property
    def shape(self):
        """(rows, feature columns + label columns), the shape of the reference's data_set."""
        return (self.n_rows, self.feats.shape[1] + self.labels.shape[1])

    def __array__(self, dtype=None, copy=None):
        """The reference's data_set (data_io.py:236-282): float64 [features | labels] rows, for
        callers that read item 5 of read_lab_fea's shared list as an array (a host copy)."""
        a = np.concatenate([self.feats.cpu().numpy().astype(np.float64),
                            self.labels.cpu().numpy().astype(np.float64)], 1)
        return a if dtype is None else a.astype(dtype)

    def finish(self):
        return self


def trim_end_index(end_index, left, right):
    """load_chunk's end_index after the context window (data_io.py:130-131)."""
    end_index = np.asarray(end_index) - left
    end_index[-1] = end_index[-1] - right
    return end_index


class PendingChunk(Chunk):
    """Item 5 of read_lab_fea's shared list: a chunk whose utterances are sorted / split and whose
    raw frames are uploading (StagedChunk, one per feature stream); the GPU half of load_chunk
    (context windows, chunk normalisation, label shift, stream stacking, frame shuffle) runs on
    finish() — which run_nn calls where the reference's loader thread shuffles, so the np.random
    draws keep the reference's order — or on first use of the device tensors.

    streams: [(StagedChunk, cw_left, cw_right, fea_name)] in fea_dict order (data_io.py:184)."""

    def __init__(self, streams, labs, lab_names, max_seq, shuffle_rng):
        self._pending = (streams, labs, list(lab_names), max_seq, shuffle_rng)
        Lm, Rm = max(l for _, l, _, _ in streams), max(r for _, _, r, _ in streams)
        cols, c = {}, 0
        for st, l, r, fname in streams:
            w = st.shape[1] * (l + r + 1)
            cols[fname] = (c, c + w)
            c += w
        super().__init__(streams[0][0].names, trim_end_index(streams[0][0].end_index, Lm, Rm), None,
                         None, cols, list(lab_names))

    def finish(self):
        if self._pending is not None:
            streams, labs, lab_names, max_seq, rng = self._pending
            self._pending = None
            ch = prepare_streams(streams, lab_names, shuffle_rng=rng)
            self._feats, self._labels = ch.feats, ch.labels
        return self

    @property
    def feats(self):
        return self.finish()._feats

    @feats.setter
    def feats(self, v):
        self._feats = v

    @property
    def labels(self):
        return self.finish()._labels

    @labels.setter
    def labels(self, v):
        self._labels = v


class StagedChunk:
    """A chunk after the host half of loading: utterances sorted / split (load_dataset) and the
    raw frames on their way to HBM — copied from pinned host memory by an asynchronous copy on a
    dedicated stream (hipMemcpyAsync underneath), so the upload of chunk k+1 overlaps the
    training of chunk k (run_nn stages the next chunk from its loader thread).

    With a Kaldi front-end (pkc.frontend.FeaFrontend: apply-cmvn / add-deltas), whole utterances
    are uploaded in their own order and pkc_feat_frontend writes the processed frames in the
    sorted / split order on the same stream."""

    def __init__(self, names, raw, lab_arrays, end_index, device, fe_args=None):
        self.names, self.lab_arrays, self.end_index = names, lab_arrays, end_index
        dev = torch.device(device)
        self.stream = torch.cuda.Stream(device=dev)
        host = [raw] + ([] if fe_args is None else list(fe_args["arrays"]))
        pinned = []
        for a in host:
            t = torch.empty(a.shape, dtype=torch.float32 if a.dtype == np.float32 else torch.int32,
                            pin_memory=True)
            t.numpy()[...] = a
            pinned.append(t)
        with torch.cuda.stream(self.stream):
            dev_t = [t.to(dev, non_blocking=True) for t in pinned]
            if fe_args is None:
                self.raw_d = dev_t[0]
            else:
                raw_src, srow, urow, ubeg, uend, unorm, norm, scales = dev_t
                Nout, Dout = fe_args["out_shape"]
                self.raw_d = torch.empty(Nout, Dout, dtype=torch.float32, device=dev)
                call("pkc_feat_frontend", ptr(raw_src), int(raw.shape[1]), Nout, ptr(srow),
                     ptr(urow), ptr(ubeg), ptr(uend), ptr(unorm), ptr(norm), fe_args["cmvn_mode"],
                     ptr(scales), fe_args["order"], fe_args["maxoff"], ptr(self.raw_d),
                     C.c_void_p(self.stream.cuda_stream))
                self._dev_inputs = dev_t
            self.done = torch.cuda.Event()
            self.done.record(self.stream)
        self.shape = tuple(self.raw_d.shape)
        self._pinned = pinned           # alive until the copy has completed (finish_chunk)


def frontend_args(fea, pieces, frontend):
    """Host tables of pkc_feat_frontend for these pieces: the utterances' raw frames in one array
    (each utterance whole, in order of first use), per-output-row source frame and utterance,
    per-utterance frame range and cmvn table index, the cmvn tables and the delta windows."""
    from .frontend import delta_scales
    keys = list(dict.fromkeys(k for k, _, _ in pieces))
    if not keys:
        raise ValueError("empty chunk: no utterance survived the feature / label / cmvn filters")
    D = fea[keys[0]].shape[1]
    uid = {k: i for i, k in enumerate(keys)}
    lens = np.array([len(fea[k]) for k in keys], dtype=np.int64)
    ubeg = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    if int(lens.sum()) >= 2 ** 31:
        raise ValueError("chunk too large for the int32 front-end row maps")
    raw = np.ascontiguousarray(np.concatenate([fea[k] for k in keys]), dtype=np.float32)
    srow = np.concatenate([np.arange(a, b) + ubeg[uid[k]] for k, a, b in pieces]).astype(np.int32)
    urow = np.concatenate([np.full(b - a, uid[k]) for k, a, b in pieces]).astype(np.int32)
    kept, norm, nidx, mode = frontend.norm_tables(keys, D)
    if kept != keys:
        raise ValueError("utterances without cmvn statistics reached the front-end")
    if mode == 0:
        norm = np.zeros((1, 2, D), np.float32)
        nidx = np.zeros(len(keys), np.int32)
    scales, maxoff = delta_scales(frontend.order, frontend.window)
    arrays = [srow, urow, ubeg.astype(np.int32), (ubeg + lens).astype(np.int32),
              nidx.astype(np.int32), norm.astype(np.float32), scales.astype(np.float32)]
    return dict(raw=raw, arrays=arrays, cmvn_mode=mode, order=frontend.order, maxoff=maxoff,
                out_shape=(len(srow), frontend.out_dim(D)))


def stage_chunk(fea, labs, max_sequence_length, device="cuda", frontend=None):
    if frontend is None:
        names, raw, lab_arrays, end_index = load_dataset(fea, labs, max_sequence_length)
        return StagedChunk(names, np.ascontiguousarray(raw, dtype=np.float32), lab_arrays,
                           end_index, device)
    # apply-cmvn writes nothing for utterances it has no statistics for: drop them before the
    # label filter / sort / split of load_dataset
    D = next(iter(fea.values())).shape[1] if fea else 0
    kept = set(frontend.norm_tables(sorted(fea), D)[0])
    fea = {k: v for k, v in fea.items() if k in kept}
    names, pieces, lab_arrays, end_index = dataset_pieces({k: len(v) for k, v in fea.items()}, labs,
                                                          max_sequence_length)
    fa = frontend_args(fea, pieces, frontend)
    return StagedChunk(names, fa["raw"], lab_arrays, end_index, device, fe_args=fa)


def prepare_chunk(fea, labs, lab_names, left, right, max_sequence_length, shuffle_rng=None,
                  device="cuda", fea_name="fea", staged=None, frontend=None):
    """data_io.load_chunk + read_lab_fea for one feature stream (data_io.py:121-145, 155-282):
    context window, chunk z-normalisation, label shift by the chunk minimum, optional frame
    shuffle (rng: the RandomState the reference's global np.random would be, seeded by run_nn).
    staged: the StagedChunk of these utterances when the loader thread already uploaded them."""
    if staged is None:
        staged = stage_chunk(fea, labs, max_sequence_length, device, frontend=frontend)
    return prepare_streams([(staged, left, right, fea_name)], lab_names, shuffle_rng=shuffle_rng,
                           device=device)


def prepare_streams(streams, lab_names, shuffle_rng=None, device="cuda"):
    """data_io.read_lab_fea over K feature streams (data_io.py:184-282), each a StagedChunk of the
    same utterances with its own context window: every stream is expanded and z-normalised over its
    OWN chunk (load_chunk, :121-145), then trimmed to the widest window — rows
    [cw_left_max - L, N - L - R - (cw_right_max - R)) of its expansion (:216-219) — and
    column-stacked in stream order (:235-240); the labels are the first stream's (:232-233), shifted
    by their chunk minimum and trimmed alike; one frame shuffle permutes the stacked rows
    (:269-270).  Each stream is written straight into its column range of one chunk matrix in HBM
    (pkc_cw_apply_rows)."""
    st0 = streams[0][0]
    names, lab_arrays, end_index = st0.names, st0.lab_arrays, st0.end_index
    N = st0.shape[0]
    for st, _, _, fname in streams[1:]:
        # data_io.py:244-253: the same sentences and end indexes in every stream
        if list(st.names) != list(names) or st.shape[0] != N or \
                not np.array_equal(np.asarray(st.end_index), np.asarray(end_index)):
            raise ValueError("feature stream %s: different sentence ids or lengths than %s (the "
                             "reference stops on this, data_io.py:244-253)" % (fname, streams[0][3]))
    Lm, Rm = max(l for _, l, _, _ in streams), max(r for _, _, r, _ in streams)
    Nout = N - Lm - Rm
    if Nout <= 0:
        raise ValueError("chunk of %d frames is shorter than the context window" % N)
    end_index = trim_end_index(end_index, Lm, Rm)
    widths = [st.shape[1] * (l + r + 1) for st, l, r, _ in streams]
    Ctot = int(sum(widths))
    lab_cols = []
    for la in lab_arrays:                      # data_io.py:137-141, then the trim of :216
        la = la - la.min()
        lab_cols.append(la[Lm:N - Rm])
    labels = np.stack(lab_cols, 1).astype(np.int32) if lab_cols else np.zeros((Nout, 0), np.int32)
    perm = None
    if shuffle_rng is not None:                # same draws as shuffling the (Nout, C) matrix rows
        perm = np.arange(Nout, dtype=np.int64)
        shuffle_rng.shuffle(perm)
        labels = labels[perm]
    dev = torch.device(device)
    cur = torch.cuda.current_stream(dev)
    s = C.c_void_p(cur.cuda_stream)
    feats = torch.empty(Nout, Ctot, dtype=torch.float32, device=dev)
    perm_d = torch.from_numpy(perm).to(dev) if perm is not None else None
    fea_cols, c0 = {}, 0
    for (st, left, right, fname), w in zip(streams, widths):
        cur.wait_event(st.done)
        raw_d = st.raw_d
        raw_d.record_stream(cur)
        D = st.shape[1]
        mean = torch.empty(w, dtype=torch.float64, device=dev)
        std = torch.empty(w, dtype=torch.float64, device=dev)
        work = torch.empty(int(L.lib().pkc_cw_stats_work_size(N, D, left, right)),
                           dtype=torch.float64, device=dev)
        call("pkc_cw_stats", ptr(raw_d), N, D, left, right, ptr(mean), ptr(std), ptr(work), s)
        call("pkc_cw_apply_rows", ptr(raw_d), N, D, left, right, ptr(mean), ptr(std), ptr(perm_d),
             Lm - left, Nout, C.c_void_p(feats.data_ptr() + 4 * c0), Ctot, s)
        fea_cols[fname] = (c0, c0 + w)
        c0 += w
    labels_d = torch.from_numpy(np.ascontiguousarray(labels)).to(dev)
    return Chunk(names, end_index, feats, labels_d, fea_cols, list(lab_names))
