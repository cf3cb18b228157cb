"""pkc.dist — chunk-level data parallelism for run_nn.

One process per GPU (torchrun / torch.distributed.run sets RANK, LOCAL_RANK, WORLD_SIZE,
MASTER_ADDR/PORT).  Every rank builds the same model from the same seeds (HCGS / pattern masks and
init are drawn from the cfg seed, core.py:41-44), loads the same chunk and trains on a disjoint
share of it:

  * frame models (MLP): the shuffled frame matrix is cut into R contiguous row ranges;
  * sequence models: the length-sorted sentences are dealt round-robin (rank r takes sentences
    r, r+R, ...), so every rank sees the same length profile and similar padded batch shapes;
  * every rank runs the same number of steps: the minimum over ranks (the reference drops the
    remainder of a chunk the same way, core.py:157-162).

Exchange per optimizer step: ONE all-reduce (SUM) of the flat fp32 gradient buffer the engine
keeps (Engine.gflat, 26.7 MB for C1/C2), over RCCL ("nccl" backend = RCCL on ROCm, xGMI links).
The engine pre-scales the loss gradient by 1/R, so the summed gradient is the gradient of the
mean of the ranks' batch losses — each rank's loss being the reference's own per-batch loss.
No other collective is on the data path.  Per chunk: the loss / err totals are summed for the
.info file, and the BatchNorm running statistics (updated locally from each rank's batches) are
averaged so the saved model is one replica.
"""
import os

import numpy as np
import torch
import torch.distributed as dist


def world():
    """(rank, world_size) of the current process group (0, 1 when not distributed)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's environment (no-op for one process).
    backend: "nccl" (RCCL) when a GPU is visible, else "gloo"."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1 or (dist.is_available() and dist.is_initialized()):
        return world()
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
    return world()


def shard_rows(n_rows, rank, ws):
    """[r0, r1) rows of a frame chunk owned by `rank` (contiguous, equal sizes, remainder dropped)."""
    per = n_rows // ws
    return rank * per, (rank + 1) * per


def shard_sentences(end_index, rank, ws):
    """Sentences of a length-sorted chunk owned by `rank`: (begin rows, lengths) int64 arrays of
    sentences rank, rank+ws, ... (end_index: cumulative sentence ends, data_io.py:81-83)."""
    e = np.asarray(end_index, dtype=np.int64)
    b = np.concatenate([[0], e[:-1]])
    sel = np.arange(rank, len(e), ws)
    return b[sel], (e - b)[sel]


def agree_min(n, device=None):
    """The minimum of an integer over all ranks (steps every rank can run)."""
    rank, ws = world()
    if ws == 1:
        return int(n)
    t = torch.tensor([int(n)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def frame_weight(rows, device=None):
    """This rank's share of the rows of the global batch (its loss scale under sequence DP: the
    padded T_r * B rows differ between ranks, so 1/R would weight a short batch's rows more than a
    long one's).  One scalar all-reduce; the engine takes a whole chunk's scales at once
    (frame_weights)."""
    rank, ws = world()
    if ws == 1:
        return 1.0
    t = torch.tensor([float(rows)], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return float(rows) / float(t.item())


def frame_weights(sent_len, B, n_batches, device=None):
    """Every batch's loss scale for this rank over a whole chunk of sequence DP: batch i of rank r
    is padded to T_r[i] = the longest of its B sentences, so its rows are T_r[i] * B and its share
    of the global batch i is T_r[i] / sum_r' T_r'[i] (see frame_weight).  The T's follow from the
    sentence lengths alone (the random left padding does not change them), so ONE all-reduce per
    chunk replaces the per-step scalar all-reduce and its host sync.  Returns float64 (n_batches,)."""
    lens = np.asarray(sent_len, dtype=np.int64)[:n_batches * B].reshape(n_batches, B)
    T = lens.max(1).astype(np.float64)
    rank, ws = world()
    if ws == 1:
        return np.ones(n_batches)
    t = torch.zeros((ws, n_batches), dtype=torch.float64, device=device)
    t[rank] = torch.from_numpy(T).to(t.device)
    dist.all_reduce(t)
    return T / t.sum(0).cpu().numpy()


def sum_scalars(vals, device=None):
    """Element-wise sum of a list of floats over ranks."""
    rank, ws = world()
    if ws == 1:
        return [float(v) for v in vals]
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return [float(v) for v in t.cpu()]


class CAbiAllReduce:
    """The same exchange through libpkc's C ABI (pkc_dp_*: RCCL communicator of its own), as a
    non-Python host would run it (include/pkc.h).  The unique id travels over the
    torch.distributed default group (any channel works)."""

    def __init__(self, device=0):
        import ctypes as C

        from . import _lib as L
        self.L, self.C = L, C
        rank, ws = world()
        nb = L.lib().pkc_dp_unique_id_bytes()
        idb = (C.c_char * nb)()
        if rank == 0:
            L.call("pkc_dp_unique_id", idb)
        if ws > 1:
            t = torch.frombuffer(bytearray(idb.raw), dtype=torch.uint8).clone()
            dist.broadcast(t, 0)
            C.memmove(idb, bytes(t.tolist()), nb)
        self.comm = C.c_void_p()
        L.call("pkc_dp_comm_init", C.byref(self.comm), ws, idb, rank, device)
        self.calls = 0

    def __call__(self, gflat, async_op=False):
        self.calls += 1
        s = torch.cuda.current_stream()
        self.L.call("pkc_dp_allreduce", self.comm, self.L.ptr(gflat), gflat.numel(),
                    self.C.c_void_p(s.cuda_stream))
        return None

    def close(self):
        if self.comm:
            self.L.call("pkc_dp_comm_destroy", self.comm)
            self.comm = self.C.c_void_p()


class GradAllReduce:
    """Callable handed to Engine.train_step(allreduce=...): sums the flat gradient buffer over all
    ranks in one collective (the engine already scaled the loss gradient by 1/R)."""

    def __init__(self, group=None):
        self.group = group
        self.calls = 0

    def __call__(self, gflat, async_op=False):
        """async_op=True returns the work handle: the collective runs on the communicator's own
        stream, overlapping the backward kernels the caller queues meanwhile, and
        handle.wait() makes the caller's current stream wait for it (the host does not block)."""
        self.calls += 1
        return dist.all_reduce(gflat, group=self.group, async_op=async_op)


class SyncBatchNorm:
    """Engine(sync_bn=SyncBatchNorm()): the MLP layers' training-mode BatchNorm statistics over
    the GLOBAL batch of all ranks (SURVEY 8e's optional SyncBN; its DP parity recipe: R ranks on a
    split global batch equal one process on the whole batch).  Per BatchNorm layer and direction
    one small all-reduce: the ranks' (n, mean, M2) column states (forward, merged in rank order by
    pkc_dense_fwd_sync_apply) and the column sums of dy, dy * xhat (backward).  Eager steps only
    (Engine.capture returns False with it)."""

    def __init__(self, group=None):
        self.group = group
        self.rank, self.world = world()
        self.calls = 0

    def __call__(self, t):
        self.calls += 1
        if self.world > 1:
            dist.all_reduce(t, group=self.group)


def average_buffers(modules, device=None):
    """Average BatchNorm running_mean / running_var over ranks (one all-reduce per chunk)."""
    rank, ws = world()
    if ws == 1:
        return
    bufs = [b for m in modules for n, b in m.named_buffers()
            if n.endswith("running_mean") or n.endswith("running_var")]
    if not bufs:
        return
    flat = torch.cat([b.detach().reshape(-1).to(device or b.device) for b in bufs])
    dist.all_reduce(flat)
    flat /= ws
    off = 0
    for b in bufs:
        n = b.numel()
        b.copy_(flat[off:off + n].view_as(b).to(b.device))
        off += n


def check_replicas(modules, device=None):
    """True when every rank holds bit-identical parameters (one max/min all-reduce of a checksum);
    run once after init: the masks and weights come from identical seeds on every rank."""
    rank, ws = world()
    if ws == 1:
        return True
    acc = torch.zeros(2, dtype=torch.float64, device=device)
    for m in modules:
        for p in m.parameters():
            v = p.detach().double().reshape(-1).to(acc.device)
            idx = torch.arange(1, v.numel() + 1, dtype=torch.float64, device=acc.device)
            acc[0] += (v * idx).sum()
            acc[1] += v.abs().sum()
    hi, lo = acc.clone(), acc.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    return bool(torch.equal(hi, lo))
