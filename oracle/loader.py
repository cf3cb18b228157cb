"""Oracle: chunk loader + Kaldi ark I/O restated in numpy (test infrastructure only).

Restates reference data_io.py:
  load_dataset   data_io.py:16-88     (filter, sort, split long utterances, re-sort, concat)
  context_window data_io.py:105-118   (np.roll concatenation, future frame block first)
  load_chunk     data_io.py:121-145   (context, end_index shift, chunk z-norm, label -= min)
  read_lab_fea   data_io.py:155-282   (streams x labels, trim to max context, column_stack, shuffle)
  write_mat      data_io.py:770-806   (Kaldi binary 'FM ' matrix, ark key prefix)
  load_counts    data_io.py:148-152
"""
import struct

import numpy as np


def load_dataset(fea, lab, max_sequence_length):
    """data_io.py:16-88 with the Kaldi pipes replaced by in-memory dicts {key: array}."""
    if lab is not None:
        lab = {k: v for k, v in lab.items() if k in fea}          # data_io.py:20-22
        fea = {k: v for k, v in fea.items() if k in lab}          # data_io.py:23-24
    names, fc, lc = [], [], []
    for k in sorted(sorted(fea.keys()), key=lambda k: len(fea[k])):  # data_io.py:34
        f = fea[k]
        l = lab[k] if lab is not None else np.zeros((f.shape[0],))
        T = len(f)
        if T > max_sequence_length > 0:                            # data_io.py:41-72
            m = max_sequence_length
            j = 0
            start = 0
            while True:
                rest = T - start
                if rest > m + m / 4:
                    fc.append(f[start:start + m]); lc.append(l[start:start + m])
                    names.append("%s_split%d" % (k, j))
                    start += m
                    j += 1
                else:
                    fc.append(f[start:]); lc.append(l[start:])
                    names.append("%s_split%d" % (k, j))
                    break
                if j >= (T + m - 1) // m:
                    break
        else:
            fc.append(f); lc.append(l); names.append(k)
    order = sorted(range(len(fc)), key=lambda i: fc[i].shape[0])   # stable, data_io.py:77-79
    fc = [fc[i] for i in order]
    lc = [lc[i] for i in order]
    end_index = np.cumsum([x.shape[0] for x in fc])
    return names, np.concatenate(fc), np.concatenate(lc), end_index


def context_window(fea, left, right):
    """data_io.py:105-118: column block b holds np.roll(fea, lag_b) with lag_b = -left+b, i.e. the
    frame t - lag_b: the first block is the *future* frame t+left ... the last is t-right."""
    N, D = fea.shape
    out = np.empty((N, D * (left + right + 1)))                   # float64, as np.empty default
    for b, lag in enumerate(range(-left, right + 1)):
        out[:, b * D:(b + 1) * D] = np.roll(fea, lag, axis=0)
    return out[left:N - right]


def load_chunk(fea, lab, left, right, max_sequence_length):
    """data_io.py:121-145."""
    names, data, labs, end_index = load_dataset(fea, lab, max_sequence_length)
    if left != 0 or right != 0:
        data = context_window(data, left, right)
    end_index = end_index - left
    end_index[-1] = end_index[-1] - right
    data = (data - np.mean(data, axis=0)) / np.std(data, axis=0)
    labs = labs - labs.min()
    labs = labs[left:-right] if right > 0 else labs[left:]
    return names, np.column_stack((data, labs)), end_index


def read_lab_fea(streams, labels, seq_model, to_do="train", max_seq_length=1000, rng=None):
    """data_io.py:155-282 for in-memory inputs.

    streams: list of (name, fea_dict, cw_left, cw_right); labels: list of (name, lab_dict).
    rng: a numpy RandomState used for the frame shuffle (global np.random in the reference,
    seeded at core.py:40 before the first read)."""
    cw_l = max(s[2] for s in streams)
    cw_r = max(s[3] for s in streams)
    fea_cols, lab_cols = {}, {}
    data_set = labs = end_index = names = None
    fea_index = 0
    for fi, (fname, fea, L, R) in enumerate(streams):
        for li, (lname, lab) in enumerate(labels):
            n, ds, end = load_chunk(fea, lab, L, R, max_seq_length)
            lab_f = ds[cw_l - L:ds.shape[0] - (cw_r - R), -1]
            ds = ds[cw_l - L:ds.shape[0] - (cw_r - R), 0:-1]
            end = end - (cw_l - L)
            end[-1] = end[-1] - (cw_r - R)
            if fi == 0 and li == 0:
                data_set, labs, end_index, names = ds, lab_f, end, n
                fea_cols[fname] = (fea_index, fea_index + ds.shape[1])
                fea_index += ds.shape[1]
            else:
                if fi == 0:
                    labs = np.column_stack((labs, lab_f))
                if li == 0:
                    data_set = np.column_stack((data_set, ds))
                    fea_cols[fname] = (fea_index, fea_index + ds.shape[1])
                    fea_index += ds.shape[1]
                assert names == n and (end_index == end).all()
    for li, (lname, _) in enumerate(labels):
        lab_cols[lname] = data_set.shape[1] + li
    data_set = np.column_stack((data_set, labs))
    if not seq_model and to_do != "forward":
        (rng if rng is not None else np.random).shuffle(data_set)   # data_io.py:269-270
    return names, end_index, fea_cols, lab_cols, data_set


# ------------------------------------------------------------------------------------------------
# Kaldi ark I/O
# ------------------------------------------------------------------------------------------------
def mat_bytes(m, key=""):
    """data_io.py:770-806 (binary 'FM '/'DM ' matrix, optional ark key)."""
    out = b""
    if key:
        out += (key + " ").encode("latin1")
    out += b"\0B"
    if m.dtype == np.float32:
        out += b"FM "
    elif m.dtype == np.float64:
        out += b"DM "
    else:
        raise TypeError(m.dtype)
    out += b"\x04" + struct.pack("<I", m.shape[0]) + b"\x04" + struct.pack("<I", m.shape[1])
    return out + np.ascontiguousarray(m).tobytes()


def parse_mat_ark(buf):
    """Binary ark of FM/DM matrices -> list of (key, ndarray) (data_io.py:645-711)."""
    out, pos = [], 0
    while pos < len(buf):
        sp = buf.index(b" ", pos)
        key = buf[pos:sp].decode("latin1")
        pos = sp + 1
        assert buf[pos:pos + 2] == b"\0B"
        hdr = buf[pos + 2:pos + 5]
        dt = {b"FM ": np.float32, b"DM ": np.float64}[hdr]
        rows = struct.unpack("<i", buf[pos + 6:pos + 10])[0]
        cols = struct.unpack("<i", buf[pos + 11:pos + 15])[0]
        pos += 15
        n = rows * cols * np.dtype(dt).itemsize
        out.append((key, np.frombuffer(buf[pos:pos + n], dtype=dt).reshape(rows, cols)))
        pos += n
    return out


def vec_int_bytes(v, key):
    """Kaldi binary int32 vector (the format read by data_io.py:431-445)."""
    v = np.asarray(v, dtype=np.int32)
    rec = np.empty(len(v), dtype=[("size", "i1"), ("value", "<i4")])
    rec["size"] = 4
    rec["value"] = v
    return (key + " ").encode("latin1") + b"\0B\x04" + struct.pack("<i", len(v)) + rec.tobytes()


def load_counts(text):
    """data_io.py:148-152 (first line '[ c1 c2 ... ]')."""
    row = text.splitlines()[0].strip().strip("[]").strip()
    return np.array([np.float32(v) for v in row.split()])


def decode_cm(blob):
    """data_io.py:729-766 (_read_compressed_mat, "CM " only): blob = bytes after "\\0BCM "."""
    gmin, grange, rows, cols = np.frombuffer(blob[:16], dtype="<f4,<f4,<i4,<i4", count=1)[0]
    ph = np.frombuffer(blob[16:16 + 8 * cols], dtype="<u2").reshape(cols, 4)
    hdr = (ph * grange * 1.52590218966964e-05 + gmin).astype(np.float32)
    data = np.frombuffer(blob[16 + 8 * cols:16 + 8 * cols + rows * cols], dtype=np.uint8)
    data = data.reshape(cols, rows)
    p0, p25, p75, p100 = (hdr[:, i:i + 1] for i in range(4))
    m = np.where(data <= 64, p0 + (p25 - p0) / 64. * data,
                 np.where(data > 192, p75 + (p100 - p75) / 63. * (data - 192),
                          p25 + (p75 - p25) / 128. * (data - 64)))
    return np.ascontiguousarray(m.T, dtype=np.float32)
