"""pkc.engine — executes the cfg [model] graph on the HIP kernels of libpkc.so.

What it replaces: core.run_nn's per-batch body (core.py:180-232) — utils.forward_model's
interpreter (utils.py:1884-2050) over MLP / liGRU / LSTM archs (neural_networks.py:245-319,
823-1112, 1523-1599), the LogSoftmax + NLLLoss + cost_err heads, autograd backward and the
per-architecture optimizer steps.

Design (MI355X-first):
  * every tensor of a step lives in preallocated HBM buffers sized for the largest batch; kernels
    take the runtime row count (T*B for sequence batches);
  * non-sequential models: a step is a fixed sequence of ~35 launches on one stream (no host sync:
    loss/err accumulate on the device), captured once into a hipGraph and replayed per batch; the
    batch is gathered from the HBM-resident chunk by a device-side batch counter;
  * sequence models: the padded (T, B, F) batch is assembled on the GPU (pkc_seq_gather) from
    host-drawn padding offsets; each recurrent layer = gate matmuls over all T*B rows (MFMA) +
    BN + the per-step time loop (pkc_rnn_fwd / pkc_rnn_bwd, one launch per step);
  * matmuls: pkc_gemm (MFMA, split-K slabs summed by the consumers); BN/act/dropout fused in
    pkc_dense_fwd/_bwd; LogSoftmax+NLL+err+dlogits fused in pkc_nll_fused; every optimizer of
    every architecture in one pkc_optim_step that also re-applies HCGS masks.
"""
import ctypes as C
import os
import random
import re
import zlib

import numpy as np
import torch

from . import _lib as L
from ._lib import call, ptr
from .cgs import kmeans_patterns

_PAT = re.compile(r"(.*)=(.*)\((.*),(.*)\)")
# split-K slab budget of a layer output (<= 8: the small-batch dense kernels sum them in
# registers); on the C2 step 4 gives 0.197 ms per step, 8 and 5 0.201, 3 0.211, 2 0.233
MAX_SPLITS = int(os.environ.get("PKC_MAX_SPLITS", "4"))
# slab budget of a layer output read by several matmul layers (the output heads' shared input:
# the 1928-wide head's dX gets 7 K-splits instead of 3).  C2, same run, frames/s: 4 -> 668-670k,
# 5 -> 674-677k, 6 -> 675-677k, 8 -> 682-683k
SLAB_BUDGET_MULTI = min(8, int(os.environ.get("PKC_SLAB_BUDGET_MULTI", "8")))
# forward Z = X W^T (0: by precision — MAX_SPLITS for bf16 operands; 8 for exact fp32, whose
# 128-row forward matmuls are bound by each workgroup's fp32 operand bytes and MFMA chain: C2 fp32
# 565k -> 578k frames/s with 8, 487k with 2, same box, profiles/r03_fp32_splits_ab.txt); an
# explicit PKC_MAX_SPLITS still caps the fp32 forward splits when PKC_MAX_SPLITS_FWD is unset
MAX_SPLITS_FWD = int(os.environ.get("PKC_MAX_SPLITS_FWD", "0"))
_FP32_FWD_SPLITS = MAX_SPLITS if "PKC_MAX_SPLITS" in os.environ else 8
# spread optimizer updates: a layer's update larger than this many parameters is cut into parts
# that ride in successive backward launches (0: one part).  Round 1 (fp32-stored operands), C2
# frames/s: 0 -> 653-657k, 1.2M -> 663k, 700k -> 666-667k, 400k-520k -> 669-671k, 250k -> 644k.
# With bf16-stored operands and the 8-column BatchNorm kernels the backward launches are shorter
# and the heads' 2M-parameter update no longer needs cutting: 500k 762-763k, 1M 768-771k,
# 2.5M (heads in one part) 768-772k, 300k 728k (profiles/r02_opt_spread_ab.txt).  Round 3, with the
# grouped launches at 4 waves per SIMD the heads' update again sets its launch's length (11.3 of
# 14.3 us, profiles/r03_launch_probe.txt): 2.5M 863-869k, 1M 874-876k, 700k 878-879k, 500k
# 874-875k (profiles/r03_opt_spread_ab.txt)
OPT_SPREAD_PARAMS = int(os.environ.get("PKC_OPT_SPREAD_PARAMS", "700000"))
# the spread updates' work items take their tensors' pointers from the launch's kernel arguments
# (pkc_opt_seg) instead of a chunk map -> descriptor -> data chain of dependent loads (0: map form)
OPT_DIRECT = os.environ.get("PKC_OPT_DIRECT", "1") != "0"
# sequence models: pinned host slots of the per-batch metadata upload, and the number of captured
# per-T step graphs kept (least recently used dropped first)
SEQ_META_SLOTS = 4
# bf16 performance mode of the sequence models (Engine prec PKC_PREC_BF16): the recurrent step
# products U h_{t-1} / dgates U^T on bf16 operand copies too (pkc_rnn_args.step_bf16; liGRU /
# LSTM / RNN layers without quantised h or LayerNorm, dense or block-sparse U).  0: exact-fp32
# steps, bf16 matmuls only.
RNN_BF16 = os.environ.get("PKC_RNN_BF16", "1") != "0"
RNN_BF16_SPARSE = os.environ.get("PKC_RNN_BF16_SPARSE", "0") != "0"     # block-sparse U too
# persistent liGRU time loops for block-sparse U in bf16 step mode (pkc_rnn_persist.hip; 0: the
# per-step launches)
RNN_PERSIST = os.environ.get("PKC_RNN_PERSIST", "1") != "0"
# quantised-h LSTM steps with U on an 8-bit (or coarser) weight grid (C5): the step products as
# exact integer sums on the bf16 MFMA (pkc_rnn_args.qh_exact) in every precision — the fp32
# products to within their own rounding; 0: the exact-fp32 chain
RNN_QH_EXACT = os.environ.get("PKC_RNN_QH_EXACT", "1") != "0"
SEQ_GRAPHS = int(os.environ.get("PKC_SEQ_GRAPHS", "512"))
# a padded length T is captured at its SEQ_CAPTURE_AFTER-th batch (eager before): real chunks have
# many one-off lengths, and a capture costs more than an eager step
SEQ_CAPTURE_AFTER = max(1, int(os.environ.get("PKC_SEQ_CAPTURE_AFTER", "2")))
# split-K dW at large frame batches (M >= this many rows): a 1024x1024 dW has only 64 128x128
# tiles, one per CU on a quarter of the chip, each a 4096-deep chain at B = 4096 (81 us); split
# 4 ways into slabs (29 us) that a slab-sum operation of the next grouped launch adds into the
# gradient (0: off)
DW_SPLIT_ROWS = int(os.environ.get("PKC_DW_SPLIT_ROWS", "1024"))
# multi-step graphs: the last launch of a step (the first layer's weight update, which needs the
# dW of the step's last matmul launch) rides in the NEXT step's first launch, beside that step's
# batch gather (PKC_OP_GATHER): one launch per step fewer; 0: off (A/B)
DEFER_TAIL = os.environ.get("PKC_DEFER_TAIL", "1") != "0"
# multi-step graphs of the B = 128 MLP step: every weight update of step k rides in step k+1's
# forward launches (the batch gather and the forward matmuls, latency-bound launches that move few
# bytes) instead of the backward launches, each before the first launch that reads its parameters
# (PKC_OPT_FWD=1; the graph's last step updates at its own end).  Measured slower: C2 886-887 k ->
# 868-870 k frames/s (profiles/r04_opt_fwd_ab.txt): the forward launches grow by more than the
# backward ones shrink, so off by default
OPT_FWD = os.environ.get("PKC_OPT_FWD", "0") != "0"
# large-batch BatchNorm backward: its statistics (sum dy, sum dy * xhat per column) in the epilogue
# of the dX matmul that produces the layer's output gradient (pkc_bn_bwd_epi), instead of a pass
# that re-reads that gradient.  Measured slower (B = 4096: 5.46-5.47 M -> 4.84-4.85 M frames/s,
# profiles/r04_bn_bwd_epi_ab.txt), so off by default (PKC_BN_BWD_EPI=1: on)
BN_BWD_EPI = os.environ.get("PKC_BN_BWD_EPI", "0") != "0"
# large-batch BatchNorm'd MLP layers: column statistics in the forward matmul's epilogue
# (pkc_gemm_colstats + pkc_dense_fwd_pre); PKC_GEMM_COLSTATS=0: matmul + stats/finalize/apply (A/B)
COLSTATS = os.environ.get("PKC_GEMM_COLSTATS", "1") != "0"
# recurrent layers' dW / dU split-K cap (1: unsplit, A/B)
REC_DW_SPLITS = int(os.environ.get("PKC_REC_DW_SPLITS", "4"))
# bf16 step mode: the recurrent weight gradients on bf16 operand copies (BF16IN; 0: fp32 staged)
REC_WGRAD_BF16 = os.environ.get("PKC_REC_WGRAD_BF16", "1") != "0"
# workgroups a layer's grouped weight-gradient launch aims at before it splits the contraction
REC_WG_TARGET = int(os.environ.get("PKC_REC_WG_TARGET", "512"))
# B <= 128 bf16 MLP layers: matmul + BatchNorm / activation / dropout in one launch
# (pkc_dense_gemm_fwd) instead of the split-K matmul + pkc_dense_fwd pair.  Same box, two
# alternating rounds: C2 0.1429 / 0.1437 ms per step fused against 0.1423 / 0.1423 for the pair
# (19 vs 24 launches per step): each workgroup of the fused form ingests all 128 rows of the input
# (256 KB at K = 1024), the pair's split-K tiles 16 KB — off by default (1: on)
FUSED_FWD = os.environ.get("PKC_FUSED_FWD", "0") != "0"
# recurrent layers: sum the output-gradient slabs before the BPTT loop (0: per step, A/B)
REC_DY_PRESUM = os.environ.get("PKC_REC_DY_PRESUM", "1") != "0"


_PAT3 = re.compile(r"(.*)=(.*)\((.*),(.*),(.*)\)")


def parse_model(text):
    """utils.py:1888-1903 line grammar: out=op(in1,in2), split at the LAST comma (greedy); a line
    whose output name starts with 'loss_gl' is re-read as out=op(in1,in2,in3) (1904-1906), and
    in3 rides in in2 as "in2,in3"."""
    rows = []
    for line in text.split("\n"):
        if not line.strip():
            continue
        row = list(_PAT.findall(line)[0])
        if row[0][:7] == "loss_gl":
            o, op, a, b, c = _PAT3.findall(line)[0]
            row = [o, op, a, b + "," + c]
        rows.append(row)
    return rows


class RegTerm:
    """One cost_l1 / cost_l2 / cost_gl line of the [model] (utils.py:24-60): a pseudo loss head
    whose per-row 'loss' is the regulariser value (pkc_reg_finalize broadcasts it)."""
    head = False

    def __init__(self, op, lam, nblk, params):
        self.op, self.lam, self.nblk, self.params = op, float(lam), nblk, params
        self.kind = L.REG_L1 if op == "cost_l1" else L.REG_L2
        self.loss_weight = 0.0

    def items(self, grads):
        """Row-slice items of every block, blocks in parameter order (gl: the torch.chunk grid
        along dim 1, then dim 0 — utils.py:49-54)."""
        items, bstart = [], [0]
        for p in self.params:
            R, Cc = p.shape[0], int(np.prod(p.shape[1:]))
            if self.op == "cost_gl":
                cs, rs = -(-Cc // self.nblk), -(-R // self.nblk)
                cgrid = [(c, min(c + cs, Cc)) for c in range(0, Cc, cs)]
                rgrid = [(r, min(r + rs, R)) for r in range(0, R, rs)]
                rects = [(r0, r1, c0, c1) for c0, c1 in cgrid for r0, r1 in rgrid]
            else:
                rects = [(0, R, 0, Cc)]
            g = grads.get(id(p))
            for r0, r1, c0, c1 in rects:
                per = max(1, 4096 // max(1, c1 - c0))
                for a in range(r0, r1, per):
                    items.append((p, g, Cc, a, min(a + per, r1), c0, c1, len(bstart) - 1))
                bstart.append(len(items))
        return items, bstart


def resolve_concat(lines, fea_cols):
    """[model] concatenate(a, b) (utils.py:2014-2016: torch.cat along the feature axis) of feature
    streams — or of earlier such concatenations — whose column ranges are adjacent in the chunk
    matrix: read_lab_fea stacks the streams in fea_dict order (data_io.py:235-240), which is the
    order the [model] first names them, so the result is the column range spanning both, a
    zero-copy view of the chunk.  Returns fea_cols with those names added."""
    cols = dict(fea_cols)
    for out, op, a, b in lines:
        if op != "concatenate":
            continue
        if a in cols and b in cols and cols[a][1] == cols[b][0]:
            cols[out] = (cols[a][0], cols[b][1])
        else:
            raise NotImplementedError("concatenate(%s,%s): only adjacent feature streams (a column "
                                      "range of the chunk) are on the pkc path" % (a, b))
    return cols


class SeqBatch(tuple):
    """(begin rows, lengths, left pads, T) of one sentence batch, plus .index: the batch's
    position in the bound chunk (its data-parallel frame weight, Engine.frame_scales)."""

    def __new__(cls, items, index):
        t = tuple.__new__(cls, items)
        t.index = index
        return t


def _f32(n, dev):
    return torch.zeros(int(max(1, n)), dtype=torch.float32, device=dev)


def _b(v):
    return str(v).strip().lower() in ("1", "true", "yes", "y", "on", "t")


def persist_geometry():
    """(waves, forward slots, BPTT slots, rows per workgroup, largest H) of the persistent loops."""
    v = [C.c_int() for _ in range(5)]
    L.lib().pkc_rnn_persist_geometry(*[C.byref(x) for x in v])
    return tuple(x.value for x in v)


def persist_plans(mask):
    """Fragment plans of the persistent liGRU loops (pkc_rnn_args.persist_*) for a static U mask
    (H x H bool, any gate): forward tiles of 16 units x the 32-wide blocks of k they read, BPTT
    tiles of 16 columns k x the 32-wide blocks of units j.  The fragments, tile by tile, are dealt
    to the waves in runs of ceil(total / waves), so every wave's per-step MFMA chain has the same
    length; a tile cut between two waves flushes from both, the second part into a spill-over tile
    (bit 18, its index in bits 19-21) that the cell update adds.  Tiles without a nonzero block take
    no slot (their products are zero).  None when the layer does not fit
    (pkc_rnn_persist_geometry)."""
    nw, nsf, nsb, _, hmax = persist_geometry()
    H = mask.shape[0]
    if H > hmax or H % 2:
        return None
    hp = -(-H // 32) * 32
    mp = np.zeros((hp, hp), dtype=bool)
    mp[:H, :H] = mask
    nt = -(-H // 16)
    fwd = mp.reshape(hp // 16, 16, hp // 32, 32).any(axis=(1, 3))[:nt]       # [unit tile][k blk]
    bwd = mp.reshape(hp // 32, 32, hp // 16, 16).any(axis=(1, 3)).T[:nt]     # [k tile][j blk]
    out = []
    for pres, nslot in ((fwd, nsf), (bwd, nsb)):
        blocks = [np.nonzero(pres[t])[0].tolist() for t in range(nt)]
        seq = [(t, b) for t in range(nt) for b in blocks[t]]
        # a run at least one tile long: a tile is cut at most once (two parts)
        run = max(1, -(-len(seq) // nw), max(len(b) for b in blocks))
        if run > nslot:
            return None
        tab = np.zeros((nw, nslot), dtype=np.int32)
        nsplit, first_wave = 0, {}
        for i, (t, b) in enumerate(seq):
            wv, f = divmod(i, run)
            first_wave.setdefault(t, wv)
            last = i + 1 == len(seq) or seq[i + 1][0] != t or (i + 1) % run == 0
            ent = t | ((b + 1) << 8) | (int(last) << 16) | (1 << 17)
            if last and wv != first_wave[t]:         # the second part of a cut tile: its own slot
                ent |= (1 << 18) | (nsplit << 19)
                nsplit += 1
            tab[wv, f] = ent
        assert nsplit < nw
        out.append(tab.reshape(-1))
    return out


def _splits(M, N, K, cap):
    return max(1, min(cap, L.lib().pkc_gemm_pick_splits(M, N, K)))


class Layer:
    """One dense layer of an MLP architecture inside the graph."""
    rec = False

    def __init__(self, arch, idx, spec, K):
        self.arch, self.idx, self.K = arch, idx, K
        self.N = spec["out"]
        self.spec = spec
        self.act = spec["act"]
        self.head = self.act == "softmax"
        self.bn = spec["bn"]
        self.drop = float(spec["drop"])
        self.W, self.b = spec["W"], spec["b"]
        self.gamma, self.beta, self.rm, self.rv = spec["gamma"], spec["beta"], spec["rm"], spec["rv"]
        self.mask = spec["mask"]
        self.src = None          # ("fea", c0, c1) or ("node", producer)
        self.consumers = []
        self.label_col = None
        self.nbt0 = int(spec["nbt"].item()) if spec.get("nbt") is not None else 0
        self.loss_weight = 0.0
        self.name = "%s.%d" % (arch, idx)
        if self.head and self.bn:
            raise NotImplementedError("%s: BatchNorm before LogSoftmax is not on the pkc path" % self.name)
        self.ln = bool(spec["ln"])                # LayerNorm between the Linear and BN / act
        self.ln_gamma, self.ln_beta = spec.get("ln_gamma"), spec.get("ln_beta")
        if self.act not in L.ACT and not self.head:
            raise NotImplementedError("%s: activation %s" % (self.name, self.act))
        self.qbits = int(spec["quant"] or 0)      # QuantizeLinear weight bits (0: nn.Linear)
        self.ibits = int(spec["inp_quant"] or 0)  # QuantizeLinear input bits (0: off)
        self.reads = 1 if self.ibits else 0       # in-place input quantisations this layer applies
        self.Wq = None

    def params(self):
        out = [(self.W, "dW", self.mask), (self.b, "db", None)]
        if self.ln:
            out += [(self.ln_gamma, "dgamma_ln", None), (self.ln_beta, "dbeta_ln", None)]
        if self.bn:
            out += [(self.gamma, "dgamma", None), (self.beta, "dbeta", None)]
        return out

    def quant_of(self, p):
        return (self.Wq, self.qbits) if (p is self.W and self.qbits) else (None, 0)


# Block-sparse U in the recurrent step kernels for static HCGS masks: "auto" (when it cuts the
# contraction), "force" (whenever the tiles fit, used by the parity tests) or "off".
RNN_SPARSE = os.environ.get("PKC_RNN_SPARSE", "auto")
# Block-sparse W matmuls (forward and dX) for static masks: "auto" (when at most this fraction of
# the 64 x 32 weight tiles holds a nonzero), "force" (any saving) or "off".
W_SPARSE = os.environ.get("PKC_W_SPARSE", "auto")
W_SPARSE_MAX_FRAC = 0.75


def ktile_table(mask, transpose, dev):
    """k-tile lists of a block-sparse matmul (include/pkc.h pkc_gemm_problem.ktiles) for a static
    (out, in) weight mask: forward Z = X W^T tiles 64 output units and lists the 32-wide input
    blocks with a nonzero; dX = dZ W (transpose) tiles 64 inputs and lists the 32-wide output
    blocks.  Returns (int32 device table [tiles, kmax + 1], kmax, kept fraction) or None."""
    m = (mask.detach() != 0)
    if transpose:
        m = m.t()
    R, K = m.shape
    nt, nk = -(-R // 64), -(-K // 32)
    pm = torch.zeros(nt * 64, nk * 32, dtype=torch.bool, device=m.device)
    pm[:R, :K] = m
    blocks = pm.view(nt, 64, nk, 32).any(3).any(1).cpu()          # [tile][k-tile]
    counts = blocks.sum(1)
    kmax = int(counts.max().item())
    frac = float(counts.sum().item()) / (nt * nk)
    if W_SPARSE == "off" or kmax >= nk or (W_SPARSE != "force" and frac > W_SPARSE_MAX_FRAC):
        return None
    tab = torch.full((nt, kmax + 1), -1, dtype=torch.int32)
    for i in range(nt):
        idx = torch.nonzero(blocks[i]).flatten()
        tab[i, 0] = len(idx)
        tab[i, 1:1 + len(idx)] = idx.to(torch.int32)
    return tab.to(dev), kmax, frac


class NormLayer(Layer):
    """An MLP's input LayerNorm / BatchNorm (dnn_use_laynorm_inp / dnn_use_batchnorm_inp,
    neural_networks.py:246-251): a node with no matmul, normalising the arch's input."""

    def __init__(self, arch, idx, spec, K):
        self.arch, self.idx, self.K, self.N = arch, idx, K, K
        self.spec = spec
        self.kind = spec["kind"]
        self.act, self.head, self.drop = "linear", False, 0.0
        self.bn, self.ln = self.kind == "bn", self.kind == "ln"
        self.gamma, self.beta = spec["gamma"], spec["beta"]
        self.ln_gamma, self.ln_beta = spec["gamma"], spec["beta"]
        self.rm, self.rv = spec.get("rm"), spec.get("rv")
        self.W = self.b = self.mask = None
        self.src, self.consumers, self.label_col = None, [], None
        self.nbt0 = int(spec["nbt"].item()) if spec.get("nbt") is not None else 0
        self.loss_weight = 0.0
        self.name = "%s.inp_%s%d" % (arch, self.kind, idx)
        self.qbits = self.ibits = self.reads = 0
        self.Wq = None

    def params(self):
        if self.ln:
            return [(self.gamma, "dgamma_ln", None), (self.beta, "dbeta_ln", None)]
        return [(self.gamma, "dgamma", None), (self.beta, "dbeta", None)]


class RecNode:
    """A whole liGRU / LSTM architecture (all its layers) as one graph node."""
    rec = True
    head = False

    def __init__(self, arch, net, K):
        self.arch, self.net, self.K = arch, net, K
        self.name = arch
        self.cell = {"lstm": L.CELL_LSTM, "gru": L.CELL_GRU, "ligru": L.CELL_LIGRU,
                     "minimalgru": L.CELL_MINGRU, "rnn": L.CELL_RNN}[net.cell]
        self.G = {L.CELL_LSTM: 4, L.CELL_GRU: 3, L.CELL_LIGRU: 2, L.CELL_MINGRU: 2,
                  L.CELL_RNN: 1}[self.cell]
        # two-phase cells: the candidate gate's U multiplies r*h (GRU) / z*h (minimalGRU)
        self.cand = {L.CELL_GRU: 2, L.CELL_MINGRU: 1}.get(self.cell)
        self.layers = net.layer_specs()
        self.N = net.out_dim
        self.src = None
        self.consumers = []
        self.loss_weight = 0.0
        self.label_col = None
        for sp in self.layers:
            if sp["act"] not in L.ACT:
                raise NotImplementedError("%s: activation %s" % (arch, sp["act"]))
            sp["nbt0"] = [int(bn.num_batches_tracked.item()) for bn in sp["bnm"]]
            sp.setdefault("qbits", 0)
            sp.setdefault("ibits", 0)
            if sp["ibits"] and sp["bidir"]:
                raise NotImplementedError("%s: input quantisation of a bidirectional layer" % arch)
        # in-place quantisations of the node's input (gate linears of layer 0)
        self.ibits = self.layers[0]["ibits"]
        self.reads = self.G if self.ibits else 0
        self.qw = {}            # id(param) -> fake-quantised copy
        self.emask = {}         # id(param) -> effective (HCGS x pattern) mask

    def params(self):
        out = []
        for li, sp in enumerate(self.layers):
            for g in range(self.G):
                W = sp["W"][g]
                wm = sp["Wmasks"][g] if sp.get("Wmasks") else sp["Wmask"]
                out.append((W, ("dW", li, g), self.emask.get(id(W), wm)))
                if sp["b"][g] is not None:
                    out.append((sp["b"][g], ("db", li, g), None))
            for g in range(self.G):
                U = sp["U"][g]
                um = sp["Umasks"][g] if sp.get("Umasks") else sp["Umask"]
                out.append((U, ("dU", li, g), self.emask.get(id(U), um)))
            if sp["bn"]:
                for g in range(self.G):
                    out.append((sp["bnm"][g].weight, ("dgamma", li, g), None))
                    out.append((sp["bnm"][g].bias, ("dbeta", li, g), None))
            if sp.get("ln"):
                out.append((sp["ln_gamma"], ("dgamma_ln", li, 0), None))
                out.append((sp["ln_beta"], ("dbeta_ln", li, 0), None))
        return out

    def quant_of(self, p):
        q = self.qw.get(id(p))
        if q is None:
            return None, 0
        return q

    def wq(self, li, kind, g):
        """The weight a GEMM / the time loop multiplies with (fake-quantised when quantised)."""
        p = self.layers[li][kind][g]
        q = self.qw.get(id(p))
        return q[0] if q is not None else p


def pattern_effective_masks(net, s):
    """Pattern masks (neural_networks.py:263-272, 876-884; sparsity.py:1112-1146) of one
    architecture: computed once, at the first layer call, from |W| of every pattern-masked weight —
    layer 0's input weights already multiplied by their HCGS mask, every other weight raw — and
    then multiplied into all of them once per layer call (L times per forward; {0,1} except on
    tied tiles).  Masks already held in ``net.pattern_mask`` (carried between chunks by run_nn,
    core.py:129-131, 304-306) are reused, as the reference does; new ones are stored there in the
    reference's structure.  Each weight's pattern set is, in order: the one carried in
    ``net.pattern``; the shared set (``pattern_kernels`` / ``pattern_from_file``); or a KMeans
    search of that weight (update_patterns, neural_networks.py:339-348, 1162-1172), stored back
    into ``net.pattern``.  Returns {id(param): HCGS x pattern^L effective mask}."""
    if not getattr(net, "if_pattern", False):
        return {}
    dev = next(net.parameters()).device
    entries = net.pattern_params()
    nl = 1 + max(e[1] for e in entries)
    store, pstore = net.pattern_mask, net.pattern
    have = all(_pm_get(store, key) is not None for key, _, _, _ in entries)
    shared = net.pattern_kernels
    if shared is None and not have and not net.can_search_patterns():
        raise NotImplementedError("%s: pattern masks need a pattern set" % net.arch_name)
    out = {}
    for key, li, p, hmask in entries:
        rows, cols = p.shape
        if have:
            pm = _pm_get(store, key).to(dev, torch.float32).contiguous()
        else:
            pre = li == 0 and hmask is not None and _is_input_weight(key)
            src = (p * hmask if pre else p).contiguous()
            pk = _pm_get(pstore, _pattern_key(key))
            if pk is not None:
                t = pk.detach().cpu().numpy() if torch.is_tensor(pk) else np.asarray(pk)
                pk = t.reshape(t.shape[0], t.shape[-2], t.shape[-1]).astype(np.float32)
            elif shared is not None:
                pk = shared
            else:                               # update_patterns: one KMeans search per weight
                pn, shape, nnz = net.pattern_search_args(li)
                pk = kmeans_patterns(src, pn, shape, nnz, random_state=net.pattern_seed)
            P, ph, pw = pk.shape
            if rows % ph or cols % pw:
                raise NotImplementedError("%s: %dx%d weight not tiled by %dx%d patterns"
                                          % (net.arch_name, rows, cols, ph, pw))
            pat = torch.from_numpy(np.ascontiguousarray(pk, dtype=np.float32)).to(dev)
            pm = torch.empty_like(p)
            call("pkc_pattern_mask", ptr(src), rows, cols, ptr(pat), P, ph, pw, ptr(pm), s)
            _pm_set(store, key, pm)
            if _pm_get(pstore, _pattern_key(key)) is None:
                _pm_set(pstore, _pattern_key(key), pat.view(P, 1, ph, pw))
        e = pm.pow(nl) if nl > 1 else pm.clone()
        out[id(p)] = e * hmask if hmask is not None else e
    return out


def _pattern_key(key):
    """net.pattern key of a net.pattern_mask key: (None, i) for an MLP layer, ('pattern_wfx', i)
    for ('pattern_mask_wfx', i) of an LSTM (neural_networks.py:1162-1172)."""
    name, i = key
    return (None if name is None else name.replace("pattern_mask_", "pattern_"), i)


def _is_input_weight(key):
    name, _ = key
    return name is None or name.startswith("pattern_mask_w")


def _pm_get(store, key):
    name, i = key
    lst = store if name is None else store.get(name, [])
    return lst[i] if i < len(lst) else None


def _pm_set(store, key, v):
    name, i = key
    lst = store if name is None else store.setdefault(name, [])
    while len(lst) <= i:
        lst.append(None)
    lst[i] = v


class Engine:
    """Training / validation executor of a [model] graph.

    nets      : {arch_name: pkc.neural_networks module} (parameters already on the device)
    arch_opts : {arch_name: configparser section} (optimizer + arch_freeze keys)
    lines     : parsed [model] lines
    fea_cols  : {fea_name: (c0, c1)} column range of each feature stream in the chunk matrix
    lab_names : ordered label names (label buffer column order)
    batch     : frames per batch (non-sequential) or sentences per batch (sequential)
    max_len   : sequential models: the longest padded batch (frames) the buffers must hold
    """

    def __init__(self, nets, arch_opts, lines, fea_cols, lab_names, batch, prec=L.PREC_FP32,
                 device="cuda", seed=0, train=True, drop_keep_in=None, grad_scale=1.0, max_len=None,
                 rnn_drop_in=None, sync_bn=None, bf16_store=None, external=False):
        self.dev = torch.device(device)
        # external: the architecture plug-in's trainable forward (pkc.plugin) — the input comes
        # from the caller, the output gradient from autograd, and the parameter / input gradients
        # go back to autograd; no loss heads, no optimizer (torch.optim steps the parameters)
        self.external = bool(external)
        self.want_dx = False
        self.nets, self.arch_opts, self.lines = nets, arch_opts, lines
        self.B = int(batch)
        self.prec = prec
        self.train = train
        self.seed = int(seed)
        self.grad_scale = float(grad_scale)    # 1/world_size under data parallelism
        # sequence DP: this rank's loss scale of every batch of the bound chunk (its share of the
        # global batch's rows, pkc.dist.frame_weights: one collective per chunk, none per step),
        # indexed by batch; None: the fixed grad_scale
        self.frame_scales = None
        # SyncBN (pkc.dist.SyncBatchNorm): the MLP layers' BatchNorm statistics over all ranks
        self.sync_bn = sync_bn
        if sync_bn is not None:
            # SyncBN covers the BatchNorm of the MLP layers (the DP parity recipe);
            # input-normalisation BatchNorms and the recurrent layers' gate BatchNorms keep
            # per-rank statistics: refuse a model whose parity would silently not hold
            for a, net in nets.items():
                if getattr(net, "seq_model", False) and any(
                        sp.get("bn") for sp in net.layer_specs()):
                    raise NotImplementedError("sync_bn: %s is recurrent with BatchNorm (its gate "
                                              "statistics are per rank)" % a)
                if any(sp.get("kind") == "bn" for sp in (net.input_norm_specs() if hasattr(net, "input_norm_specs") else [])):
                    raise NotImplementedError("sync_bn: %s has an input BatchNorm (per-rank "
                                              "statistics)" % a)
        self.prof = None                       # profile mode: list of per-launch events
        fea_cols = resolve_concat(lines, fea_cols)
        self.F = max(c1 for _, c1 in fea_cols.values())
        self.fea_cols = fea_cols
        self.lab_names = list(lab_names)
        self.nlab = len(self.lab_names)
        self.seq = any(getattr(n, "seq_model", False) for n in nets.values())
        if self.seq and not max_len:
            raise ValueError("sequence models need max_len")
        self.max_len = int(max_len) if self.seq else 1
        self.Mmax = self.B * self.max_len
        self.M = self.Mmax                     # runtime rows of the current batch
        self.T = self.max_len
        self.drop_keep_in = drop_keep_in or {}
        self.rnn_drop_in = rnn_drop_in or {}
        # the step form is fixed when the engine is built (module switches read once, here)
        self.rnn_bf16_sparse = RNN_BF16_SPARSE
        self._build_graph()
        self._alloc()
        self._build_masks()
        self._build_wtiles()
        self._build_kmaps()
        self._build_optim()
        self._build_reg()
        self._build_h16(bf16_store)
        self.graph = None
        self.graph_opt = None
        self.graph_multi, self.steps_per_graph = None, 1
        self.graph_tail = None
        self.seq_graphs = None                 # sequence models: padded T -> captured step
        self.steps_done = 0
        self.skip_labels = set()
        self.n_launches = 0                    # libpkc launches issued (or captured) so far
        self.graph_launches_per_step = None    # of the multi-step graph (capture)
        # grid-synchronised time loops (pkc_rnn_persist_form 2) that gave up waiting for a peer
        # workgroup (every spin is bounded; the loop then ends and sets its timeout word): summed
        # on the device after each such launch, raised at the next host sync (loss_values /
        # chunk_totals) instead of passing on a half-computed layer
        self.loop_fail = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self._loop_forms = {}

    # ------------------------------------------------------------------ graph construction
    def _build_graph(self):
        self.nodes, produced = [], {}
        for out, op, a, b in self.lines:
            if op != "compute":
                continue
            net = self.nets[a]
            net.check_supported()
            if b in self.fea_cols:
                src = ("fea",) + tuple(self.fea_cols[b])
                K = src[2] - src[1]
            elif b in produced:
                src = ("node", produced[b])
                K = produced[b].N
            else:
                raise ValueError("input %s of %s is neither a feature nor a produced output" % (b, a))
            if getattr(net, "seq_model", False):
                # (src may be a feed-forward node over the T*B rows, e.g. the MLP_layers_first ->
                # liGRU of TIMIT_mfcc_fbank_fmllr_liGRU_best.cfg: its gradient is the recurrent
                # layer 0's dX slabs, handed over in _rec_bwd)
                # input LayerNorm / BatchNorm over the T*B rows (neural_networks.py:1511-1516 ...)
                for i, spec in enumerate(net.input_norm_specs() if hasattr(net, "input_norm_specs")
                                         else []):
                    nl = NormLayer(a, i, spec, K)
                    nl.src = src
                    if src[0] == "node":
                        src[1].consumers.append(nl)
                    self.nodes.append(nl)
                    src = ("node", nl)
                node = RecNode(a, net, K)
                node.src = src
                if src[0] == "node":
                    if getattr(src[1], "rec_consumer", None) is not None:
                        raise NotImplementedError("%s: read by two recurrent archs" % src[1].name)
                    src[1].rec_consumer = node      # its gradient: the rec layer-0 dX slabs
                self.nodes.append(node)
                produced[out] = node
                continue
            prev = src
            for i, spec in enumerate(net.input_norm_specs() if hasattr(net, "input_norm_specs")
                                     else []):
                nl = NormLayer(a, i, spec, K)
                nl.src = prev
                if prev[0] == "node":
                    prev[1].consumers.append(nl)
                self.nodes.append(nl)
                prev = ("node", nl)
            for i, spec in enumerate(net.layer_specs()):
                lay = Layer(a, i, spec, K)
                lay.src = prev
                if prev[0] == "node":
                    prev[1].consumers.append(lay)
                self.nodes.append(lay)
                prev = ("node", lay)
                K = lay.N
                if lay.head and i != len(net.dnn_lay) - 1:
                    raise NotImplementedError("softmax only as the last layer of an MLP")
            produced[out] = prev[1]
        scal, self.err_layer = {}, None
        for out, op, a, b in self.lines:
            if op == "cost_nll":
                lay = produced[a]
                if not lay.head:
                    raise NotImplementedError("cost_nll on a non-LogSoftmax output %s" % a)
                col = self.lab_names.index(b)
                if lay.label_col is not None and lay.label_col != col:
                    raise NotImplementedError("one head with two label streams")
                lay.label_col = col
                scal[out] = {lay: 1.0}
            elif op == "cost_err":
                lay = produced[a]
                col = self.lab_names.index(b)
                if lay.label_col is None:
                    lay.label_col = col
                if lay.label_col != col:
                    raise NotImplementedError("cost_err label differs from the head's cost_nll label")
                self.err_layer = lay
            elif op == "mult_constant":
                scal[out] = {k: w * float(b) for k, w in scal[a].items()}
            elif op == "sum":
                d = dict(scal[a])
                for k, w in scal[b].items():
                    d[k] = d.get(k, 0.0) + w
                scal[out] = d
            elif op in ("cost_l1", "cost_l2", "cost_gl"):
                # utils.py:1954-1991: 0 when the first arch applies guided HCGS, else
                # lambda * sum of norms over the dim>1 parameters of archs without
                # skip_regularization (every CGS cfg but TIMIT_CGS/*L1*, *groupLasso* sets it)
                nets = list(self.nets.values())
                params, masks = [], []
                for arch, net in self.nets.items():
                    if getattr(nets[0], "apply_guided_hcgs", False):
                        break                   # the whole term is 0 (utils.py:1962)
                    if getattr(net, "skip_regularization", False):
                        continue
                    for pn, p in net.named_parameters():
                        if p.dim() > 1:
                            if "mask" in pn.split(".")[-1]:
                                # the mask Parameters are in the sum and in the optimizer, so the
                                # reference trains them; supported while they are not multiplied
                                # into W (guided masks before apply_guided_hcgs, which regenerates
                                # them at chunk end anyway)
                                if not (pn.startswith("ghcgs") and not net.apply_guided_hcgs):
                                    raise NotImplementedError(
                                        "%s over an applied mask Parameter %s.%s (the reference "
                                        "then trains the mask it multiplies in)" % (op, arch, pn))
                                masks.append((p, arch))
                            params.append(p)
                if getattr(nets[0], "apply_guided_hcgs", False) or not params:
                    scal[out] = {}
                    continue
                if op == "cost_gl":
                    if "," not in b:
                        raise NotImplementedError("cost_gl needs an output named loss_gl* "
                                                  "(utils.py:1904-1906)")
                    lam, nblk = b.split(",")
                    term = RegTerm(op, lam, int(nblk), params)
                else:
                    term = RegTerm(op, b, 0, params)
                term.masks = masks
                scal[out] = {term: 1.0}
            elif op in ("compute", "concatenate"):     # (concatenate: resolve_concat)
                continue
            else:
                raise NotImplementedError("[model] operation %s is not on the pkc path" % op)
        for n in self.nodes:
            if getattr(n, "rec_consumer", None) is not None and n.consumers:
                # its gradient would be the recurrent dX slabs AND the other consumers' slabs
                raise NotImplementedError("%s: read by a recurrent arch and by other archs" % n.name)
        self.produced = produced
        self.heads = [l for l in self.nodes if l.head]
        if self.train and "loss_final" not in scal and not self.external:
            raise ValueError("[model] has no loss_final")
        for lay, w in scal.get("loss_final", {}).items():
            lay.loss_weight = w
        self.reg_terms = [t for t in scal.get("loss_final", {}) if isinstance(t, RegTerm)
                          and t.loss_weight != 0.0]
        if self.err_layer is None and self.heads:
            self.err_layer = self.heads[0]
        for lay in self.nodes:
            if lay.head and lay.label_col is None:
                lay.label_col = -1
        self.layers = [n for n in self.nodes if not n.rec]     # dense layers (compat)
        self._build_quant()

    def _build_quant(self):
        """Input fake-quantisation chains (quantized_modules.py:99-119, applied through `.data` at
        :211-212): each quantising consumer of a tensor re-quantises its CURRENT value in place, so
        the consumers of one tensor see versions q1, q2, ... in model order, a non-quantising
        consumer sees the version current when it runs, and every weight gradient taken against
        that tensor uses the final version (autograd saved the same tensor object)."""
        self.qsrc = {}
        for n in self.nodes:
            key = ("fea", n.src[1], n.src[2]) if n.src[0] == "fea" else id(n.src[1])
            ent = self.qsrc.setdefault(key, dict(bits=0, Q=0, src=n.src))
            n.qkey, n.qv0 = key, ent["Q"]
            if n.reads:
                if ent["bits"] not in (0, n.ibits):
                    raise NotImplementedError("%s: two input-quantisation widths on one tensor" % n.name)
                ent["bits"] = n.ibits
                ent["Q"] += n.reads
        for key, ent in self.qsrc.items():
            if not ent["Q"] or ent["src"][0] != "node":
                continue
            P = ent["src"][1]
            # a quantised-in-place activation output changes the saved result only where autograd
            # differentiates through it (tanh/sigmoid/elu with no dropout in between)
            if not P.rec and P.act not in ("relu", "linear", "leaky_relu") and P.drop == 0.0:
                raise NotImplementedError("%s: %s output quantised in place by a consumer" %
                                          (P.name, P.act))
    def _alloc(self):
        M, dev = self.Mmax, self.dev
        self.cap = MAX_SPLITS if self.seq else None
        self.ctr = torch.zeros(2, dtype=torch.int64, device=dev)      # batch counter + done word
        self.x = _f32(M * self.F, dev)
        self.labs = torch.zeros(M * max(1, self.nlab), dtype=torch.int32, device=dev)
        for n in self.nodes:
            if n.rec:
                self._alloc_rec(n)
                continue
            N, K = n.N, n.K
            n.scap = self.cap or _splits(M, N, K, MAX_SPLITS_FWD or
                                         (_FP32_FWD_SPLITS if self.prec == L.PREC_FP32 else MAX_SPLITS))
            n.zslab = _f32(n.scap * M * N, dev) if n.W is not None else None
            if n.ln:
                n.ln_y, n.ln_xhat = _f32(M * N, dev), _f32(M * N, dev)
                n.ln_stat, n.dz_ln = _f32(2 * M, dev), _f32(M * N, dev)
            n.out = n.ln_y if (n.ln and n.W is None) else _f32(M * N, dev)
            n.xhat = None if n.head else _f32(M * N, dev)
            n.keep = torch.zeros(M * N, dtype=torch.uint8, device=dev) if n.drop > 0 else None
            n.save_mean = _f32(N, dev)
            n.save_invstd = _f32(N, dev)
            n.dz = _f32(M * N, dev)
            n.work = _f32(L.lib().pkc_dense_work_size(M, N), dev)
            if self.sync_bn is not None and n.bn and not n.head and n.W is not None:
                n.bn_states = _f32(self.sync_bn.world * 3 * N, dev)     # ranks' (n, mean, M2)
                n.bn_sums = _f32(2 * N, dev)                           # sum dy, sum dy * xhat
            n.sdw = self._dw_splits(N, K) if n.W is not None else 1
            n.dwslab = _f32(n.sdw * N * K, dev) if n.sdw > 1 else None
            if n.qbits:
                n.Wq = torch.zeros_like(n.W)
            if n.head:
                n.row_loss = _f32(M, dev)
                n.row_err = _f32(M, dev)
        for key, ent in self.qsrc.items():
            if not ent["Q"]:
                continue
            src = ent["src"]
            if src[0] == "fea":
                if src[1] != 0 or src[2] != self.F:
                    raise NotImplementedError("input quantisation of one of several feature streams")
                width = self.F
            else:
                width = src[1].N
            ent["width"] = width
            ent["buf"] = _f32(ent["Q"] * M * width, dev)
            ent["work"] = _f32(256, dev)
        for n in self.nodes:
            cap = 0
            for c in n.consumers:
                # an input norm (no matmul) writes its input gradient into one slab
                c.sxcap = 1 if c.W is None else (self.cap or _splits(
                    M, n.N, c.N, SLAB_BUDGET_MULTI if len(n.consumers) > 1 else MAX_SPLITS))
                cap += c.sxcap
            n.gslab = _f32(cap * M * n.N, dev) if cap else None
        self.needs_grad = {}
        for n in reversed(self.nodes):
            rc = getattr(n, "rec_consumer", None)
            self.needs_grad[n] = self.external or (n.head and n.loss_weight != 0.0) or any(
                self.needs_grad[c] for c in n.consumers) or (rc is not None and self.needs_grad[rc])
        # all gradients in ONE flat buffer (a single RCCL all-reduce under data parallelism)
        plist = [(n, p, key, m) for n in self.nodes for (p, key, m) in n.params()]
        self.gflat = _f32(sum(p.numel() for _, p, _, _ in plist), dev)
        off = 0
        self.grads = {}
        self.grad_off = {}
        self.param_grads = []                  # [(parameter, its gradient view of gflat)]
        for n, p, key, m in plist:
            self.grad_off.setdefault(n, off)
            g = self.gflat[off:off + p.numel()].view_as(p)
            self.param_grads.append((p, g))
            off += p.numel()
            if isinstance(key, tuple):
                n.lbuf[key[1]][key[0]][key[2]] = g
            else:
                setattr(n, key, g)
        self.loss_heads = [l for l in self.heads if l.label_col >= 0]
        if self.loss_heads:
            if self.err_layer not in self.loss_heads:
                raise NotImplementedError("err head without labels")
            terms = self.loss_heads + self.reg_terms
            for t in self.reg_terms:
                t.row_loss = _f32(M, dev)
            self.n_loss_terms = len(terms)
            self.loss_out = _f32(2 + len(terms), dev)
            self.loss_acc = _f32(2, dev)
            ptrs = np.array([l.row_loss.data_ptr() for l in terms], dtype=np.uint64)
            self.loss_ptrs = torch.from_numpy(ptrs.view(np.int64)).to(dev)
            self.loss_w = torch.tensor([l.loss_weight for l in terms], dtype=torch.float32,
                                       device=dev)
        if self.seq:
            self.seq_meta = torch.zeros(4 * self.B, dtype=torch.int64, device=dev)
            # host side of the per-batch metadata upload: a ring of pinned slots, each reused only
            # after the copy that read it has run (its event), so the upload never waits on the
            # device queue (the reference's per-batch host round trip, core.py:186-214)
            self.meta_ring = [torch.zeros(4 * self.B, dtype=torch.int64).pin_memory()
                              for _ in range(SEQ_META_SLOTS)]
            self.meta_ev = [None] * SEQ_META_SLOTS
            self.meta_k = 0
        if self.external:
            self.ext_dx = _f32(M * self.F, dev)   # dL/dx of the caller's input

    def _dw_splits(self, N, K):
        """K-splits of a dense layer's dW = dz^T X (contraction over the M batch rows): enough
        128x128 tiles x splits for ~256 workgroups at large batches, at most 4, >= 256 rows each."""
        M = self.Mmax
        if self.seq or DW_SPLIT_ROWS <= 0 or M < DW_SPLIT_ROWS:
            return 1
        tiles = -(-N // 128) * -(-K // 128)
        return max(1, min(4, -(-256 // tiles), M // 256))

    def _build_h16(self, want):
        """bf16 storage of the MLP matmul operands (PKC_PREC_BF16IN): the producers write a bf16
        copy beside each fp32 tensor a matmul reads — the gathered batch (pkc_batch_gather), a
        layer's output (pkc_dense_fwd out_bf16), its gradient dz (pkc_dense_bwd dz_bf16, the heads'
        dlogits_bf16) and W (the optimizer's bout) — rounded exactly as the PREC_BF16 matmuls round
        the fp32 values when they stage them, so the results are the same while every workgroup
        pulls half the operand bytes.  bf16_store=None: on unless PKC_BF16_STORE=0 (A/B).  Only
        for bf16 MLP steps without in-place weight pruning or input fake-quantisation (their
        operands change outside the producers above)."""
        if want is None:
            want = os.environ.get("PKC_BF16_STORE", "1") != "0"
        self.h16 = (bool(want) and self.prec == L.PREC_BF16 and not self.seq and not self.prune_list
                    and not any(ent["Q"] for ent in self.qsrc.values()))
        self.x_h = None
        for n in self.nodes:
            n.W_h = n.out_h = n.dz_h = None
            n.f32_dead = n.dz_scratch = False
        self.scratch_dz = set()
        self.dead_out = set()
        if not self.h16:
            return
        M, dev, bf = self.Mmax, self.dev, torch.bfloat16
        mm = [n for n in self.nodes if not n.rec and n.W is not None and not n.qbits]
        if any(n.src[0] == "fea" for n in mm):
            self.x_h = torch.zeros(M * self.F, dtype=bf, device=dev)
        keep_f32 = os.environ.get("PKC_F32_OUT", "0") != "0"
        for n in mm:
            n.W_h = torch.zeros(n.W.numel(), dtype=bf, device=dev)
            if not n.head and any(c in mm for c in n.consumers):
                n.out_h = torch.zeros(M * n.N, dtype=bf, device=dev)
                # every consumer reads the bf16 copy (forward and dW operands): a training step
                # stores no fp32 output for this layer (eval passes still do; PKC_F32_OUT=1: A/B)
                # ... only when every consumer has the whole bf16 path: a LayerNorm'd consumer
                # keeps no bf16 dz (its dW then runs in fp32 on the fp32 output), nor does a
                # consumer that needs no gradient
                n.f32_dead = (not keep_f32 and not n.ln
                              and all(c in mm and not c.ln and self.needs_grad[c]
                                      for c in n.consumers)
                              and not any(getattr(c, "qv0", 0) or getattr(c, "reads", 0)
                                          for c in n.consumers))
            if self.needs_grad[n] and not n.ln:
                n.dz_h = torch.zeros(M * n.N, dtype=bf, device=dev)
        # every matmul of the step has bf16 operand copies (so every launch runs PKC_PREC_BF16IN):
        # a BatchNorm body layer's fp32 dz is then only scratch of its own backward passes and the
        # final gradient is stored as the bf16 copy alone (pkc_dense_bwd_args.dz_scratch)
        full = all(m in mm and not m.ln for m in self.nodes if m.W is not None)
        for n in mm:
            n.dz_scratch = bool(full and not keep_f32 and not n.head and n.bn
                                and n.dz_h is not None)
            if n.dz_scratch:
                self.scratch_dz.add(n.dz.data_ptr())
            if n.f32_dead:
                self.dead_out.add(n.out.data_ptr())
        for e in self.opt_entries:
            nd = e["node"]
            if nd is not None and getattr(nd, "W_h", None) is not None and e["p"] is nd.W:
                e["bout"] = nd.W_h
        if self.opt_entries:
            self._upload_opt_desc(step_inc=1)
        self.refresh_bf16()

    def refresh_bf16(self):
        """Re-cast the bf16 weight copies from the fp32 weights (after the weights changed outside
        the optimizer, which keeps them current itself)."""
        s = self._stream()
        for n in self.nodes:
            if getattr(n, "W_h", None) is not None:
                call("pkc_cast_bf16", ptr(n.W), ptr(n.W_h), n.W.numel(), s)

    def _alloc_rec(self, n):
        M, dev, B, T = self.Mmax, self.dev, self.B, self.max_len
        G = n.G
        n.lbuf = []
        K = n.K
        for sp in n.layers:
            H = sp["H"]
            B2 = 2 * B if sp["bidir"] else B
            D = 2 * H if sp["bidir"] else H
            lb = dict(K=K, H=H, B2=B2, D=D,
                      zslab=_f32(MAX_SPLITS * M * H, dev), wpre=_f32(G * M * H, dev),
                      xhat=_f32(G * M * H, dev), sm=_f32(G * H, dev), si=_f32(G * H, dev),
                      work=_f32(L.lib().pkc_dense_work_size(M, H), dev),
                      hs=_f32((T + 1) * B2 * H, dev),
                      cs=_f32((T + 1) * B2 * H, dev) if n.cell == L.CELL_LSTM else None,
                      rh=_f32(T * B2 * H, dev) if n.cand is not None else None,
                      gates=_f32(G * T * B2 * H, dev), y=_f32(M * D, dev),
                      drop=_f32(B2 * H, dev), dgates=_f32(G * T * B2 * H, dev),
                      dpre=_f32(G * M * H, dev), dz=_f32(G * M * H, dev),
                      rwork=_f32(8 * B2 * H, dev), ut=_f32(G * H * H, dev),
                      dx=_f32(G * MAX_SPLITS * M * K, dev),
                      dW=[None] * G, db=[None] * G, dU=[None] * G, dgamma=[None] * G,
                      dbeta=[None] * G, dgamma_ln=[None], dbeta_ln=[None])
            if sp.get("ln"):
                lb.update(ln_xhat=_f32(T * B2 * H, dev), ln_stat=_f32(2 * T * B2, dev),
                          ln_g=_f32(T * B2 * H, dev), ln_pg=_f32(2 * H, dev))
            if (self.prec == L.PREC_BF16 and RNN_BF16 and not sp.get("ln") and not sp["ibits"]
                    and n.cell in (L.CELL_LIGRU, L.CELL_LSTM, L.CELL_RNN)):
                bf = torch.bfloat16            # bf16 operand copies of the step products
                lb.update(hs_h=torch.zeros((T + 1) * B2 * H, dtype=bf, device=dev),
                          U_h=torch.zeros(G * H * H, dtype=bf, device=dev),
                          ut_h=torch.zeros(G * H * H, dtype=bf, device=dev),
                          dgates_h=torch.zeros(G * T * B2 * H, dtype=bf, device=dev))
                if REC_WGRAD_BF16:            # bf16 operand copies of the weight gradients
                    lb.update(dz_h=torch.zeros(G * M * H, dtype=bf, device=dev),
                              xw_h=torch.zeros(M * K, dtype=bf, device=dev))
            if sp["ibits"]:
                lb["hq"] = _f32((T + 1) * B2 * H, dev)      # q4(h_{t-1}) per step
                # exact bf16 copies of the grid U (QX path: LSTM, h on <= 16 bits, no LayerNorm —
                # the max|h| partials it quantises with are the cell's h before an LN rewrite)
                if (RNN_QH_EXACT and 0 < sp["qbits"] <= 8 and sp["ibits"] <= 16
                        and not sp.get("ln") and n.cell == L.CELL_LSTM):
                    lb["U_hq"] = torch.zeros(G * H * H, dtype=torch.bfloat16, device=dev)
                if n.lbuf:                                   # layers >= 1: q1..qG of y_{l-1}
                    lb["xq"] = _f32(G * M * K, dev)
                    lb["qwork"] = _f32(256, dev)
            if sp["qbits"]:
                for g in range(G):
                    for p in (sp["W"][g], sp["U"][g]):
                        n.qw[id(p)] = (torch.zeros_like(p), sp["qbits"])
            n.lbuf.append(lb)
            K = D
        # split-K slabs of the weight gradients dW = dz^T x (H x K over the T*B rows) and dU (H x H
        # over the T*B2 rows): every gate's dW and dU of a layer run in ONE grouped launch, split
        # over the contraction only when that launch has too few tiles to fill the chip
        # (_rec_wgrads); room for every problem's slabs at the cap
        need = (max(n.G * REC_DW_SPLITS * (lb["H"] * lb["K"] + lb["H"] * lb["H"]) for lb in n.lbuf)
                if REC_DW_SPLITS > 1 else 0)
        n.rslab = _f32(need, dev) if need else None
        # dL/dy of a layer summed over its producers' slabs once, before the serial BPTT loop
        # (whose per-step epilogue would otherwise read every slab at every step)
        n.dysum = _f32(M * max(lb["D"] for lb in n.lbuf), dev) if REC_DY_PRESUM else None
        n.out = n.lbuf[-1]["y"]

    def _build_masks(self):
        """Pattern masks folded with the HCGS masks into one effective mask per parameter that the
        optimizer epilogue applies (see pattern_effective_masks)."""
        eff = {}
        for net in self.nets.values():
            eff.update(pattern_effective_masks(net, self._stream()))
        for n in self.nodes:
            if n.rec:
                for li, sp in enumerate(n.layers):
                    for p in list(sp["W"]) + list(sp["U"]):
                        if id(p) in eff:
                            n.emask[id(p)] = eff[id(p)]
            elif n.W is not None and id(n.W) in eff:
                n.mask = eff[id(n.W)]

    def _build_wtiles(self):
        """Block-sparse W (north_star: HCGS / pattern masks in the matmuls; HCGS.py:24-28,
        neural_networks.py:258, 858-861): the forward and dX matmuls of a weight with a static
        mask (no magnitude pruning, whose zeros move) skip the 64 x 32 weight tiles that are all
        zero.  Masked entries stay exactly zero (masks applied at build and in every optimizer
        update), so the skipped products are exact zeros and the sums are the dense ones.  dW
        stays dense: the reference's optimizer also updates (and keeps state for) masked entries."""
        self.wtiles = {}
        for n in self.nodes:
            if n.rec:
                for li, sp in enumerate(n.layers):
                    if sp.get("prune") is not None:
                        continue
                    for p, key, m in n.params():
                        if m is not None and key[0] == "dW" and key[1] == li:
                            self.wtiles[id(p)] = (ktile_table(m, False, self.dev),
                                                  ktile_table(m, True, self.dev))
            elif n.W is not None and n.mask is not None and n.spec.get("prune") is None:
                self.wtiles[id(n.W)] = (ktile_table(n.mask, False, self.dev),
                                        ktile_table(n.mask, True, self.dev))

    def _wt(self, W, dx):
        t = self.wtiles.get(id(W))
        return t[1 if dx else 0] if t is not None else None

    def _build_kmaps(self):
        """Block-sparse U for static HCGS masks (liGRU / LSTM; no prune, pattern or quantised h,
        whose zeros move): per step-kernel tile, the 16-wide contraction blocks that hold a
        nonzero of the mask (pkc_rnn_args.kmap_*).  The optimizer keeps masked entries at zero, so
        skipping the other blocks changes only the order of the fp32 sums."""
        for n in self.nodes:
            if not n.rec or n.cell not in (L.CELL_LIGRU, L.CELL_LSTM):
                continue
            for sp, lb in zip(n.layers, n.lbuf):
                lb["kmap_fwd"] = lb["kmap_bwd"] = None
                if RNN_SPARSE == "off" or sp.get("prune") is not None or sp["ibits"]:
                    continue
                um = [sp["Umasks"][g] if sp.get("Umasks") else sp["Umask"] for g in range(n.G)]
                if any(m is None or id(U) in n.emask for m, U in zip(um, sp["U"])):
                    continue
                H = lb["H"]
                nb = -(-H // 16)
                rowp, pres = [], []
                for m in um:
                    mb = torch.zeros(nb * 16, nb * 16, device=self.dev)
                    mb[:H, :H] = (m.detach().reshape(H, H) != 0).float()
                    rowp.append(mb.view(nb * 16, nb, 16).amax(2) > 0)          # [row][col blk]
                    pres.append(mb.view(nb, 16, nb, 16).amax(dim=(1, 3)) > 0)  # [row blk][col blk]
                NU = 16 // n.G
                nt = -(-H // NU)
                acc = torch.zeros(nt * NU, nb, dtype=torch.bool, device=self.dev)
                for rp in rowp:
                    acc[:H] |= rp[:H]
                fwd = acc.view(nt, NU, nb).any(1)                   # [tile][k blk]
                # BPTT tile (gate g, columns k-block kt) reads the row blocks j with a nonzero
                bwd = torch.stack([p_.t() for p_ in pres])          # [g][kt][j blk]
                dense_s = 16 if H <= 256 else 32 if H <= 512 else 48 if H <= 768 else 64 if H <= 1024 else 128

                def table(presence, rows):
                    kept = int(presence.sum(-1).max().item())
                    S = next((c for c in (16, 32, 64) if c >= kept), None)
                    if S is None or (RNN_SPARSE != "force" and S >= dense_s):
                        return None, 0
                    tab = torch.full((rows, S), -1, dtype=torch.int32)
                    pc = presence.reshape(rows, -1).cpu()
                    for i in range(rows):
                        idx = torch.nonzero(pc[i]).flatten()
                        tab[i, :len(idx)] = idx.to(torch.int32)
                    return tab.to(self.dev), S

                lb["kmap_fwd"], lb["kmap_s_fwd"] = table(fwd, nt)
                lb["kmap_bwd"], lb["kmap_s_bwd"] = table(bwd, n.G * nb)
                lb["persist_fwd"] = lb["persist_bwd"] = None
                if (RNN_PERSIST and n.cell == L.CELL_LIGRU and self.prec == L.PREC_BF16
                        and lb.get("hs_h") is not None):
                    union = torch.zeros(H, H, dtype=torch.bool, device=self.dev)
                    for m in um:
                        union |= m.detach().reshape(H, H) != 0
                    plans = persist_plans(union.cpu().numpy())
                    if plans is not None:
                        lb["persist_fwd"], lb["persist_bwd"] = (torch.from_numpy(p_).to(self.dev)
                                                                for p_ in plans)

    def _build_optim(self):
        """One pkc_opt_tensor per parameter that receives a gradient (utils.py:1833-1881)."""
        self.opt_entries = []
        self._host_maps, self._seg_keep = {}, {}
        for n in self.nodes:
            if not self.needs_grad[n] or self.external:
                continue
            o = self.arch_opts[n.arch]
            if _b(o.get("arch_freeze", "False")):
                continue
            for p, key, m in n.params():
                if isinstance(key, tuple):
                    g = n.lbuf[key[1]][key[0]][key[2]]
                else:
                    g = getattr(n, key)
                q, qb = n.quant_of(p)
                self.opt_entries.append(dict(arch=n.arch, p=p, g=g, mask=m, o=o, q=q, qbits=qb,
                                             s1=torch.zeros_like(p), s2=None, s3=None, step=0,
                                             node=n))
        # mask Parameters trained by a regulariser term only (their gradient is the term's)
        seen = {id(e["p"]) for e in self.opt_entries}
        for t in getattr(self, "reg_terms", []):
            for p, arch in t.masks:
                o = self.arch_opts[arch]
                if id(p) in seen or _b(o.get("arch_freeze", "False")) or not self.train:
                    continue
                seen.add(id(p))
                self.opt_entries.append(dict(arch=arch, p=p, g=torch.zeros_like(p), mask=None, o=o,
                                             q=None, qbits=0, s1=torch.zeros_like(p), s2=None,
                                             s3=None, step=0, node=None, reg_only=True))
        for e in self.opt_entries:
            kind = e["o"]["arch_opt"]
            if kind == "rmsprop" and (float(e["o"]["opt_momentum"]) > 0):
                e["s3"] = torch.zeros_like(e["p"])
            if kind == "rmsprop" and _b(e["o"]["opt_centered"]):
                e["s2"] = torch.zeros_like(e["p"])
            if kind == "adam":
                e["s2"] = torch.zeros_like(e["p"])
                if _b(e["o"]["opt_amsgrad"]):
                    e["s3"] = torch.zeros_like(e["p"])
        self.static_opt = all(
            e["o"]["arch_opt"] == "rmsprop" or
            (e["o"]["arch_opt"] == "sgd" and float(e["o"]["opt_momentum"]) == 0.0)
            for e in self.opt_entries)
        n = len(self.opt_entries)
        self.node_opt = {}
        if n:
            self.opt_nchunks, self.opt_map = self._chunk_map(range(n))
            # per-layer work lists: the layer's update can run as soon as its gradients are done
            for nd in self.nodes:
                idx = [i for i, e in enumerate(self.opt_entries) if e["node"] is nd]
                if idx:
                    self.node_opt[nd] = self._chunk_map(idx) + (idx,)
            self.opt_desc = torch.zeros(n * C.sizeof(L.OptTensor), dtype=torch.uint8, device=self.dev)
            self._upload_opt_desc(step_inc=1)
        # magnitude pruning (quantized_modules.py:15-28): recomputed from |W| before every
        # forward, after the HCGS / pattern masks (neural_networks.py:256-278, 858-896)
        self.prune_list = []
        for n_ in self.nodes:
            if n_.rec:
                for li, sp in enumerate(n_.layers):
                    if sp.get("prune") is not None:
                        for p in list(sp["W"]) + list(sp["U"]):
                            self.prune_list.append((p, float(sp["prune"])) + n_.quant_of(p))
            elif n_.W is not None and n_.spec.get("prune") is not None:
                self.prune_list.append((n_.W, float(n_.spec["prune"])) + n_.quant_of(n_.W))
        self.prune_work = (torch.zeros(L.lib().pkc_prune_work_size(), dtype=torch.uint8,
                                       device=self.dev) if self.prune_list else None)
        self.apply_weight_masks(self._stream())

    def apply_weight_masks(self, s):
        """The reference multiplies the masks into W in place (and QuantizeLinear clamps W to
        [-1, 1]) before every forward (neural_networks.py:256-278, 858-896;
        quantized_modules.py:207-222); the optimizer epilogue keeps that true between steps, so
        the Engine does it once here; the external mode (torch.optim steps the weights) before
        every forward.  Then prune, then fake-quantise the copy the GEMMs multiply with."""
        pruned = {id(t[0]) for t in self.prune_list}
        for n_ in self.nodes:
            for p, key, m in n_.params():
                q, qb = n_.quant_of(p)
                if id(p) in pruned:
                    if m is not None:
                        call("pkc_apply_mask", ptr(p), ptr(m), p.numel(), C.c_float(0.0), s)
                    call("pkc_prune", ptr(p), p.numel(), C.c_double(self._perc(p)), None,
                         ptr(self.prune_work), s)
                    m = None
                if m is not None or qb:
                    call("pkc_apply_mask", ptr(p), ptr(m), p.numel(), C.c_float(1.0 if qb else 0.0), s)
                if qb:
                    call("pkc_fakequant_weight", ptr(p), ptr(q), p.numel(), qb, s)

    def _perc(self, p):
        return next(t[1] for t in self.prune_list if t[0] is p)

    def _prune_kernels(self, s):
        """After the optimizer: each pruned weight re-thresholded at its percentile (and its
        fake-quantised copy refreshed)."""
        for p, perc, q, qb in self.prune_list:
            self._k("prune %d" % p.numel(), 0, 4.0 * p.numel() * 7, "pkc_prune", ptr(p), p.numel(),
                    C.c_double(perc), None, ptr(self.prune_work), s)
            if qb:
                self._k("fakequant_weight", 0, 8.0 * p.numel(), "pkc_fakequant_weight", ptr(p),
                        ptr(q), p.numel(), qb, s)

    def _chunk_map(self, idx):
        """(n_chunks, device map) of pkc_optim_step work items over the entries idx (tensor ids
        index the full descriptor array)."""
        idx = list(idx)
        if not idx:
            return 0, None
        sizes = (C.c_int64 * len(idx))(*[self.opt_entries[i]["p"].numel() for i in idx])
        nch = L.lib().pkc_optim_chunks(sizes, len(idx), None, 0)
        cmap = (C.c_int32 * (2 * nch))()
        L.lib().pkc_optim_chunks(sizes, len(idx), cmap, nch)
        m = np.frombuffer(cmap, dtype=np.int32).copy().reshape(-1, 2)
        m[:, 0] = np.asarray(idx, dtype=np.int32)[m[:, 0]]
        dev = torch.from_numpy(m.reshape(-1)).to(self.dev)
        self._host_maps[dev.data_ptr()] = m
        return nch, dev

    def _opt_segs(self, cmap, b, e):
        """Direct form of work items [b, e) of a chunk map (pkc_opt_seg runs: one per tensor, the
        pointers passed in the launch's kernel arguments), or None (PKC_OPT_DIRECT=0)."""
        if not OPT_DIRECT:
            return None
        key = (cmap.data_ptr(), b, e)
        segs = self._seg_keep.get(key)
        if segs is not None:           # step-invariant: built once per (map, range)
            return segs
        m = self._host_maps[cmap.data_ptr()][b:e]
        runs = []
        for ti, c in m:
            if runs and runs[-1][0] == ti and runs[-1][1] + runs[-1][2] == c:
                runs[-1][2] += 1
            else:
                runs.append([int(ti), int(c), 1])
        segs = (L.OptSeg * len(runs))()
        for k, (ti, c0, nc) in enumerate(runs):
            ent = self.opt_entries[ti]
            kind, o = ent["o"]["arch_opt"], ent["o"]
            sg = segs[k]
            sg.tensor, sg.chunk0, sg.nchunks = ti, c0, nc
            sg.p, sg.g = ent["p"].data_ptr(), ent["g"].data_ptr()
            keeps_s1 = kind != "sgd" or float(o.get("opt_momentum", "0")) != 0.0
            sg.s1 = ent["s1"].data_ptr() if keeps_s1 else None
            sg.s2 = ent["s2"].data_ptr() if ent["s2"] is not None else None
            sg.s3 = ent["s3"].data_ptr() if ent["s3"] is not None else None
            sg.mask = ent["mask"].data_ptr() if ent["mask"] is not None else None
            sg.qout = ent["q"].data_ptr() if ent["qbits"] else None
            sg.bout = ent["bout"].data_ptr() if ent.get("bout") is not None else None
            sg.n = ent["p"].numel()
        self._seg_keep[key] = segs
        return segs

    def _upload_opt_desc(self, step_inc):
        n = len(self.opt_entries)
        arr = (L.OptTensor * n)()
        for i, e in enumerate(self.opt_entries):
            o = e["o"]
            kind = o["arch_opt"]
            t = arr[i]
            t.p, t.g = e["p"].data_ptr(), e["g"].data_ptr()
            t.s1 = e["s1"].data_ptr()
            t.s2 = e["s2"].data_ptr() if e["s2"] is not None else None
            t.s3 = e["s3"].data_ptr() if e["s3"] is not None else None
            t.mask = e["mask"].data_ptr() if e["mask"] is not None else None
            t.n = e["p"].numel()
            t.kind = L.OPT[kind]
            t.lr = float(o["arch_lr"])
            t.wd = float(o.get("opt_weight_decay", "0"))
            t.momentum = float(o.get("opt_momentum", "0"))
            t.dampening = float(o.get("opt_dampening", "0"))
            t.alpha = float(o.get("opt_alpha", "0.99"))
            t.eps = float(o.get("opt_eps", "1e-8"))
            if kind == "adam":
                b1, b2 = [float(v) for v in o["opt_betas"].split(",")]
                t.beta1, t.beta2 = b1, b2
                t.amsgrad = _b(o["opt_amsgrad"])
            t.nesterov = _b(o.get("opt_nesterov", "False"))
            t.centered = _b(o.get("opt_centered", "False"))
            t.clampv = 1.0 if e["qbits"] else 0.0
            t.qout = e["q"].data_ptr() if e["qbits"] else None
            t.qbits = e["qbits"]
            t.bout = e["bout"].data_ptr() if e.get("bout") is not None else None
            t.step = e["step"] + step_inc
            if kind == "sgd" and e.get("has_buf"):
                t.step = max(t.step, 2)   # torch SGD starts buf = g only when it has no buffer
        host = torch.frombuffer(bytearray(C.string_at(arr, C.sizeof(arr))), dtype=torch.uint8)
        self.opt_desc.copy_(host)

    def set_lr(self, arch, lr):
        for e in self.opt_entries:
            if e["arch"] == arch:
                e["o"] = dict(e["o"], arch_lr=str(lr))
        if self.opt_entries:
            self._upload_opt_desc(step_inc=1)

    # ------------------------------------------------------------------ chunk binding
    def bind_chunk(self, feats, labels, n_rows, end_index=None, sentences=None):
        """feats: (N, F) fp32 device tensor (row stride >= F); labels: (N, nlab) int32 device;
        end_index: cumulative utterance ends (sequence models); sentences: optional (begin rows,
        lengths) subset of them (a data-parallel rank's share, pkc.dist.shard_sentences)."""
        assert feats.dtype == torch.float32 and labels.dtype == torch.int32
        assert feats.shape[1] >= self.F and labels.shape[1] == self.nlab
        key = (feats.data_ptr(), feats.stride(0), labels.data_ptr())
        if self.seq_graphs is not None and key != getattr(self, "_chunk_key", None):
            self.seq_graphs.clear()            # the captured gathers read the old chunk
            self.seq_seen = {}
        self._chunk_key = key
        self.chunk_feats, self.chunk_labels = feats, labels
        if self.seq:
            if sentences is None:
                e = np.asarray(end_index, dtype=np.int64)
                sentences = (np.concatenate([[0], e[:-1]]), e - np.concatenate([[0], e[:-1]]))
            self.sent_beg = np.asarray(sentences[0], dtype=np.int64)
            self.sent_len = np.asarray(sentences[1], dtype=np.int64)
            self.n_batches = len(self.sent_beg) // self.B           # core.py:157-159
            self.snt = 0
        else:
            self.n_batches = int(n_rows) // self.B                  # core.py:161-162
        self.ctr.zero_()
        if self.loss_heads:
            self.loss_acc.zero_()

    def next_seq_batch(self, rng=None):
        """core.py:183-200: the next B sentences, padded to the longest with a random number of
        leading zeros (python random.randint, drawn in the reference's order)."""
        rng = rng or random
        i0 = self.snt
        begs = self.sent_beg[i0:i0 + self.B]
        lens = self.sent_len[i0:i0 + self.B]
        T = int(lens.max())
        if T > self.max_len:
            raise ValueError("batch of %d frames exceeds max_len %d" % (T, self.max_len))
        lefts = np.array([rng.randint(0, T - int(l)) for l in lens], dtype=np.int64)
        self.batch_i = i0 // self.B
        self.snt += self.B
        return SeqBatch((begs.astype(np.int64), lens.astype(np.int64), lefts, T), self.batch_i)

    # ------------------------------------------------------------------ launch helpers
    @staticmethod
    def _stream():
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def _k(self, label, flops, nbytes, fn, *args):
        """Launch one libpkc entry point; in profile mode bracket it with events."""
        if label in self.skip_labels:     # measurement only (step_cost_of)
            return
        self.n_launches += 1
        if self.prof is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            call(fn, *args)
            e1.record()
            self.prof.append((label, fn, float(flops), float(nbytes), e0, e1, args))
        else:
            call(fn, *args)

    def _src(self, n):
        if n.src[0] == "fea":
            return self.x.data_ptr() + 4 * n.src[1], self.F
        return n.src[1].out.data_ptr(), n.src[1].N

    def _src_h(self, n):
        """bf16 copy of n's (unquantised) matmul input, same leading dimension as _src, or None."""
        if not self.h16:
            return None
        if n.src[0] == "fea":
            return None if self.x_h is None else self.x_h.data_ptr() + 2 * n.src[1]
        P = n.src[1]
        return None if getattr(P, "out_h", None) is None else P.out_h.data_ptr()

    @staticmethod
    def _h_variant(pr, A, B):
        """The same problem with bf16 operand pointers (PKC_PREC_BF16IN), or None."""
        if A is None or B is None:
            return None
        q = L.GemmProblem.from_buffer_copy(pr)
        q.A, q.B = A, B
        return q

    def _version(self, n, v):
        """(pointer, ld) of version v of n's input tensor (0: as produced, k: after k in-place
        input quantisations)."""
        if v == 0:
            return self._src(n)
        ent = self.qsrc[n.qkey]
        w = ent["width"]
        return ent["buf"].data_ptr() + 4 * (v - 1) * self.M * w, w

    def _final_version(self, n):
        """The value autograd saw for n's input at backward time (dW operand)."""
        return self._version(n, self.qsrc[n.qkey]["Q"])

    def _quant_chain(self, n, s):
        """Materialise q1..qQ of n's input once, at its first quantising consumer."""
        if not n.reads or n.qv0 != 0:
            return
        ent = self.qsrc[n.qkey]
        x_ptr, _ = self._src(n)
        nel = self.M * ent["width"]
        self._k("fakequant_input x%d" % ent["Q"], 0, 4.0 * nel * (ent["Q"] + 2),
                "pkc_fakequant_input", C.c_void_p(x_ptr), ptr(ent["buf"]), nel, ent["bits"],
                ent["Q"], ptr(ent["work"]), s)

    # ------------------------------------------------------------------ forward
    def _gather(self, s, batch=None):
        if not self.seq:
            M = self.M
            self._k("batch_gather", 0, 8.0 * M * self.F, "pkc_batch_gather", ptr(self.chunk_feats),
                    self.chunk_feats.stride(0), self.F, ptr(self.chunk_labels), self.nlab, self.B,
                    self.n_batches, ptr(self.ctr), ptr(self.x), ptr(self.labs),
                    0 if self.loss_heads else 1, ptr(self.x_h), s)
            return
        T = batch[3]
        mp = self.seq_meta.data_ptr()
        self._k("seq_gather", 0, 8.0 * T * self.B * self.F, "pkc_seq_gather", ptr(self.chunk_feats),
                self.chunk_feats.stride(0), self.F, ptr(self.chunk_labels), self.nlab,
                C.c_void_p(mp), C.c_void_p(mp + 8 * self.B), C.c_void_p(mp + 8 * self.B + 4 * self.B),
                self.B, T, ptr(self.x), ptr(self.labs), s)

    def _place_fwd_opt(self, ops):
        """Slots of the previous step's weight updates in this step's forward: the gather launch
        (key None) or a matmul launch (key: its first node), each update before the launch that
        first reads its node's parameters, greedily balanced by bytes (8 operations per launch)."""
        order, first, nprob = [None], {}, {None: 1}
        i = 0
        while i < len(self.nodes):
            n = self.nodes[i]
            if n.rec or n.W is None:
                first.setdefault(n, order[-1])
                i += 1
                continue
            grp = [n]
            while (n.head and i + len(grp) < len(self.nodes) and not self.nodes[i + len(grp)].rec
                   and self.nodes[i + len(grp)].head and self.nodes[i + len(grp)].src == n.src):
                grp.append(self.nodes[i + len(grp)])
            for g in grp:
                first[g] = n
            order.append(n)
            nprob[n] = len(grp)
            i += len(grp)
        pos = {k: j for j, k in enumerate(order)}
        load = {k: [0.0, nprob[k]] for k in order}     # bytes, operations of each launch
        slots = {}
        # tightest deadline first: an update may ride in any launch before its node's own
        for n, op in sorted(ops, key=lambda t: pos.get(first.get(t[0]), 0)):
            last = pos[first[n]] - 1 if first.get(n) is not None else 0
            cands = [k for k in order[:max(1, last + 1)] if load[k][1] < 8]
            k = min(cands, key=lambda c: load[c][0]) if cands else None
            load[k][0] += op[2]
            load[k][1] += 1
            slots.setdefault(k, []).append(op)
        return slots

    def _upload_seq_meta(self, batch):
        """[B x int64 begin rows][B x int32 lengths][B x int32 left pads] of a sentence batch into
        seq_meta: an asynchronous copy from a pinned ring slot, ordered on the stream before the
        step's gather (no host synchronisation per batch)."""
        begs, lens, lefts, _ = batch[:4]
        k = self.meta_k % SEQ_META_SLOTS
        self.meta_k += 1
        if self.meta_ev[k] is not None:
            self.meta_ev[k].synchronize()        # the copy that last read this slot has run
        host = self.meta_ring[k].numpy()
        host[:self.B] = begs
        h32 = host[self.B:].view(np.int32)
        h32[:self.B] = lens
        h32[self.B:2 * self.B] = lefts
        self.seq_meta.copy_(self.meta_ring[k], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.meta_ev[k] = ev

    def _gather_op(self):
        """The frame batch gather as an operation of a grouped launch (PKC_OP_GATHER)."""
        M = self.M
        p = L.GemmProblem(kind=L.OP_GATHER, M=self.B, N=self.F, A=self.chunk_feats.data_ptr(),
                          lda=self.chunk_feats.stride(0), B=self.chunk_labels.data_ptr(),
                          ldb=self.nlab, C=self.x.data_ptr(), slab_stride=self.n_batches,
                          X1=self.ctr.data_ptr(), X2=self.labs.data_ptr(),
                          X3=self.x_h.data_ptr() if self.x_h is not None else None)
        return ("gather", 0.0, 8.0 * M * self.F, p)

    def _fwd_problem(self, n):
        """(label, flops, bytes, GemmProblem) of a dense layer's forward matmul Z = X W^T."""
        M = self.M
        a_ptr, lda = self._version(n, n.qv0 + n.reads)
        kt = self._wt(n.W, False)
        sf = 1 if kt is not None else _splits(M, n.N, n.K, n.scap)
        n.sf = sf
        W = n.Wq if n.qbits else n.W
        pr = L.GemmProblem(a_kcontig=1, b_kcontig=1, M=M, N=n.N, K=n.K, splits=sf, A=a_ptr, lda=lda,
                           B=W.data_ptr(), ldb=n.K, C=n.zslab.data_ptr(), ldc=n.N,
                           slab_stride=M * n.N)
        d = 1.0
        if kt is not None:
            pr.ktiles, pr.kmax, d = kt[0].data_ptr(), kt[1], kt[2]
        prh = self._h_variant(pr, self._src_h(n) if not (n.qv0 + n.reads) else None,
                              n.W_h.data_ptr() if n.W_h is not None else None)
        return ("fwd %dx%dx%d%s" % (M, n.N, n.K, " sparse %.2f" % d if kt is not None else ""),
                2.0 * M * n.N * n.K * d, 4.0 * (M * n.K + n.N * n.K * d + sf * M * n.N), pr,
                None if prh is None else (2.0 * (M * n.K + n.N * n.K * d) + 4.0 * sf * M * n.N, prh))

    def _gemms(self, probs, s):
        """Launch matmul problems: one pkc_gemm, or pkc_gemm_grouped for several (<= 8 each).
        A launch whose matmuls all have bf16 operand copies (a 5th tuple item: (bytes, problem))
        runs on them (PKC_PREC_BF16IN); its other operations are precision-neutral."""
        for i in range(0, len(probs), 8):
            # dX problems lead the launch: at a workgroup offset that is a multiple of 8 (the
            # preceding dX grids have 16k-wide tile rows), tile j of a 1024-column dX runs on XCD
            # j % 8 — the XCD whose BatchNorm-backward workgroups read that tile's slabs
            # (pkc_dense.hip col_group<2>)
            part = sorted(probs[i:i + 8], key=lambda q: 0 if q[0].startswith("dX") else 1)
            gem = [q for q in part if q[3].kind == L.OP_GEMM]
            prec = self.prec
            if gem and all(len(q) > 4 and q[4] is not None for q in gem):
                prec = L.PREC_BF16IN
                part = [(q[0], q[1]) + tuple(q[4]) if len(q) > 4 and q[4] is not None else q[:4]
                        for q in part]
            else:
                part = [q[:4] for q in part]
                sd = getattr(self, "scratch_dz", None)
                if sd and any(q[3].A in sd or q[3].B in sd for q in part):
                    raise RuntimeError("fp32 matmul on a bf16-only gradient: %s"
                                       % [q[0] for q in part])
                do = getattr(self, "dead_out", None)
                if do and any(q[3].kind == L.OP_GEMM and (q[3].A in do or q[3].B in do)
                              for q in part):
                    raise RuntimeError("fp32 matmul on a layer output stored as bf16 only: %s"
                                       % [q[0] for q in part])
            if len(part) == 1 and part[0][3].kind == L.OP_GEMM and not part[0][3].ktiles:
                lab, fl, nb, p = part[0]
                self._k("gemm_" + lab, fl, nb, "pkc_gemm", prec, p.a_kcontig, p.b_kcontig,
                        p.M, p.N, p.K, C.c_void_p(p.A), p.lda, C.c_void_p(p.B), p.ldb,
                        C.c_void_p(p.C), p.ldc, p.splits, p.slab_stride, s)
            else:
                arr = (L.GemmProblem * len(part))(*[q[3] for q in part])
                self._k("gemm_group[" + ", ".join(q[0] for q in part) + "]",
                        sum(q[1] for q in part), sum(q[2] for q in part), "pkc_gemm_grouped",
                        prec, arr, len(part), s)

    def _dense_fwd(self, n, s, train):
        self._quant_chain(n, s)
        prob = self._fwd_problem(n)
        if self._fused_fwd(n, prob, s, train):
            return
        if train and self._colstats_fwd(n, prob, s):
            return
        self._gemms([prob], s)
        self._fwd_epilogue(n, s, train)

    def _colstats_fwd(self, n, prob, s):
        """Large-batch BatchNorm'd MLP layer in training: the forward matmul writes the BatchNorm
        column partials of its 128- or 64-row tiles in its epilogue (pkc_gemm_colstats) and
        pkc_dense_fwd_pre merges them and applies, so no statistics pass re-reads z.  One slab
        only; sequence models keep the stats-pass blocking their recurrent lifecycle tests are
        pinned to.  Returns False when not taken."""
        if not (COLSTATS and n.bn and not n.ln and not n.head and n.W is not None and not self.seq
                and self.M > 128 and getattr(n, "bn_states", None) is None):
            return False
        lab, fl, nb, p = prob[:4]
        if p.splits != 1 or p.ktiles:
            return False
        prec = self.prec
        if len(prob) > 4 and prob[4] is not None:
            prec, (nb, p) = L.PREC_BF16IN, prob[4]
        rows = L.lib().pkc_gemm_colstats_ok(prec, p.a_kcontig, p.b_kcontig, p.M, p.N, p.K,
                                            C.c_void_p(p.A), p.lda, C.c_void_p(p.B), p.ldb)
        if rows <= 0:
            return False
        self._k("gemm_colstats " + lab, fl, nb + 8.0 * p.N * -(-p.M // rows), "pkc_gemm_colstats",
                prec, p.a_kcontig, p.b_kcontig, p.M, p.N, p.K, C.c_void_p(p.A), p.lda,
                C.c_void_p(p.B), p.ldb, C.c_void_p(p.C), p.ldc, ptr(n.b), ptr(n.work), s)
        self._fwd_epilogue(n, s, True, pre_rows=rows)
        return True

    def _fwd_epilogue(self, n, s, train, out=None, pre_rows=0):
        """The layer's epilogue launch (BN/act/dropout, or a head's LogSoftmax/NLL); with `out`
        the head's NllArgs are only filled in (for a grouped launch).  pre_rows: the BatchNorm
        column partials are already in n.work at that blocking (pkc_gemm_colstats)."""
        M = self.M
        if n.W is None:                      # input normalisation: no matmul in front
            x_ptr, ldx = self._src(n)
            if ldx != n.N:
                raise NotImplementedError("%s: input normalisation of one of several feature "
                                          "streams" % n.name)
            n.sf = 1
            zp, sf, zs, bias = x_ptr, 1, 0, None
        else:
            zp, sf, zs, bias = n.zslab.data_ptr(), n.sf, M * n.N, n.b.data_ptr()
        if n.ln:
            self._k("layernorm_fwd N=%d" % n.N, 0, 4.0 * M * n.N * (sf + 3), "pkc_layernorm_fwd", M,
                    n.N, sf, C.c_void_p(zp), zs, C.c_void_p(bias) if bias else None, ptr(n.ln_gamma),
                    ptr(n.ln_beta), C.c_float(1e-6), ptr(n.ln_y), ptr(n.ln_xhat), ptr(n.ln_stat), s)
            zp, sf, zs, bias = n.ln_y.data_ptr(), 1, 0, None
            if n.W is None:
                return                       # out aliases ln_y
        if n.head:
            has_lab = n.label_col >= 0
            a = L.NllArgs(M=M, N=n.N, nslab=sf, zslab=zp, slab_stride=zs, bias=bias,
                          labels=(self.labs.data_ptr() + 4 * n.label_col) if has_lab else None,
                          label_stride=self.nlab, weight=n.loss_weight * self.grad_scale,
                          logp=n.out.data_ptr(), log_prior=None,
                          dlogits=(n.dz_ln if n.ln else n.dz).data_ptr() if (train and has_lab)
                          else None,
                          row_loss=n.row_loss.data_ptr(), row_err=n.row_err.data_ptr(),
                          dlogits_bf16=n.dz_h.data_ptr() if (train and has_lab and n.dz_h is not None)
                          else None)
            if out is not None:
                C.memmove(C.byref(out), C.byref(a), C.sizeof(a))
                return
            self._k("nll_fused N=%d" % n.N, 0, 4.0 * M * n.N * (sf + 2), "pkc_nll_fused",
                    C.byref(a), s)
            return
        a = self._dense_fwd_args(n, train, zp, sf, zs, bias)
        if train and n.bn and getattr(n, "bn_states", None) is not None:
            # SyncBN: this rank's column state into its row of bn_states, all-reduce (gather),
            # merge + apply
            R, r = self.sync_bn.world, self.sync_bn.rank
            n.bn_states.zero_()
            self._k("dense_fwd_stats N=%d" % n.N, 0, 4.0 * M * n.N * (sf + 1), "pkc_dense_fwd_stats",
                    C.byref(a), ptr(n.work), C.c_void_p(n.bn_states.data_ptr() + 4 * r * 3 * n.N), s)
            self.sync_bn(n.bn_states)
            self._k("dense_fwd_sync_apply N=%d" % n.N, 0, 4.0 * M * n.N * 3,
                    "pkc_dense_fwd_sync_apply", C.byref(a), ptr(n.work), ptr(n.bn_states), R, s)
            return
        if pre_rows:
            self._k("dense_fwd_pre N=%d" % n.N, 0, 4.0 * M * n.N * 3, "pkc_dense_fwd_pre",
                    C.byref(a), ptr(n.work), pre_rows, s)
            return
        self._k("dense_fwd N=%d" % n.N, 0, 4.0 * M * n.N * (sf + 2), "pkc_dense_fwd",
                C.byref(a), ptr(n.work), s)

    def _dense_fwd_args(self, n, train, zp, sf, zs, bias):
        """pkc_dense_fwd_args of a dense layer's epilogue (BN / act / dropout)."""
        M = self.M
        keep_in = self.drop_keep_in.get(n.name)
        return L.DenseFwdArgs(
            M=M, N=n.N, nslab=sf, zslab=zp, slab_stride=zs, bias=bias,
            norm=(L.NORM_BN_TRAIN if train else L.NORM_BN_EVAL) if n.bn else L.NORM_NONE,
            gamma=n.gamma.data_ptr(), beta=n.beta.data_ptr(),
            running_mean=n.rm.data_ptr(), running_var=n.rv.data_ptr(),
            momentum=0.05, eps=1e-5, save_mean=n.save_mean.data_ptr(),
            save_invstd=n.save_invstd.data_ptr(), act=L.ACT[n.act],
            drop_p=n.drop if train else 0.0, seed=self.seed,
            step_ctr=self.ctr.data_ptr(), stream_id=zlib.crc32(n.name.encode()),
            keep_in=keep_in.data_ptr() if keep_in is not None else None,
            keep_out=n.keep.data_ptr() if (n.keep is not None and train) else None,
            xhat=n.xhat.data_ptr(), count_n=0,
            out=None if (train and getattr(n, "f32_dead", False)
                         and getattr(n, "bn_states", None) is None) else n.out.data_ptr(),
            out_bf16=n.out_h.data_ptr() if n.out_h is not None else None)

    def _fused_fwd(self, n, prob, s, train, riding=()):
        """A BatchNorm'd hidden layer at M <= 128 rows with bf16 products: matmul and epilogue in
        ONE launch (pkc_dense_gemm_fwd: each workgroup a 128 x 16 column strip over the full
        contraction, so its BatchNorm statistics are local) instead of a split-K matmul writing
        slabs + the pkc_dense_fwd launch.  Returns False when not taken (exact-fp32 / compensated
        precisions, block-sparse W, LayerNorm, SyncBN, operations riding in the forward launch)."""
        if not (FUSED_FWD and self.prec == L.PREC_BF16 and self.M <= 128 and not n.head
                and n.W is not None and not n.ln and not riding
                and getattr(n, "bn_states", None) is None):
            return False
        lab, fl, nb, p = prob[:4]
        if p.ktiles:
            return False
        prec = L.PREC_BF16
        if len(prob) > 4 and prob[4] is not None:
            prec, (nb, p) = L.PREC_BF16IN, prob[4]
        if not L.lib().pkc_dense_gemm_fwd_ok(prec, p.M, p.N, p.K, C.c_void_p(p.A), p.lda,
                                             C.c_void_p(p.B), p.ldb):
            return False
        n.sf = 1
        a = self._dense_fwd_args(n, train, None, 1, 0, n.b.data_ptr())
        self._k("fused_fwd %dx%dx%d" % (p.M, p.N, p.K), fl, nb - 4.0 * p.splits * p.M * p.N +
                4.0 * p.M * p.N * 2, "pkc_dense_gemm_fwd", prec, C.c_void_p(p.A), p.lda,
                C.c_void_p(p.B), p.ldb, p.K, C.byref(a), s)
        return True

    def _rnn_args(self, n, li, train, T):
        sp, lb = n.layers[li], n.lbuf[li]
        H = lb["H"]
        a = L.RnnArgs()
        a.cell, a.T, a.B, a.H, a.bidir = n.cell, T, self.B, H, int(sp["bidir"])
        a.act, a.train = L.ACT[sp["act"]], int(train)
        a.wpre = lb["wpre"].data_ptr()
        for g in range(n.G):
            a.U[g] = n.wq(li, "U", g).data_ptr()
        if sp["ibits"]:
            a.qbits, a.hq = sp["ibits"], lb["hq"].data_ptr()
        a.drop_p = float(sp["drop"])
        a.seed = self.seed
        a.step_ctr = self.ctr.data_ptr()
        a.stream_id = zlib.crc32(("%s.%d" % (n.arch, li)).encode())
        din = self.rnn_drop_in.get((n.arch, li))
        a.drop_mask_in = din.data_ptr() if din is not None else None
        a.drop_mask = lb["drop"].data_ptr()
        a.hs = lb["hs"].data_ptr()
        a.cs = lb["cs"].data_ptr() if lb["cs"] is not None else None
        a.rh = lb["rh"].data_ptr() if lb["rh"] is not None else None
        a.gates = lb["gates"].data_ptr()
        a.y = lb["y"].data_ptr()
        a.dgates = lb["dgates"].data_ptr()
        a.work = lb["rwork"].data_ptr()
        a.ut = lb["ut"].data_ptr()
        if lb.get("kmap_fwd") is not None:
            a.kmap_fwd, a.kmap_s_fwd = lb["kmap_fwd"].data_ptr(), lb["kmap_s_fwd"]
        if lb.get("kmap_bwd") is not None:
            a.kmap_bwd, a.kmap_s_bwd = lb["kmap_bwd"].data_ptr(), lb["kmap_s_bwd"]
        # (block-sparse U keeps the fp32 steps: C3's 16-row tiles over 16-wide blocks measured
        # 16.6 vs 16.1 us per step and layer with bf16 operands, profiles/r04_rnn_bf16_ab.txt)
        persist = lb.get("persist_fwd") is not None
        if lb.get("hs_h") is not None and (self.rnn_bf16_sparse or persist or (
                lb.get("kmap_fwd") is None and lb.get("kmap_bwd") is None)):
            a.step_bf16 = 1
            a.hs_h, a.ut_h, a.dgates_h = (lb["hs_h"].data_ptr(), lb["ut_h"].data_ptr(),
                                          lb["dgates_h"].data_ptr())
            for g in range(n.G):
                a.U_h[g] = lb["U_h"].data_ptr() + 2 * g * H * H
            if persist:
                a.persist_fwd, a.persist_bwd = (lb["persist_fwd"].data_ptr(),
                                                lb["persist_bwd"].data_ptr())
                a.persist_kb = persist_geometry()[1]
        if lb.get("U_hq") is not None:
            a.qh_exact = 1
            for g in range(n.G):
                a.U_h[g] = lb["U_hq"].data_ptr() + 2 * g * H * H
        if sp.get("ln"):
            a.ln_gamma, a.ln_beta, a.ln_eps = sp["ln_gamma"].data_ptr(), sp["ln_beta"].data_ptr(), 1e-6
            a.ln_xhat, a.ln_stat = lb["ln_xhat"].data_ptr(), lb["ln_stat"].data_ptr()
            a.ln_g = lb["ln_g"].data_ptr()
            if lb["dgamma_ln"][0] is not None:
                a.ln_dgamma, a.ln_dbeta = lb["dgamma_ln"][0].data_ptr(), lb["dbeta_ln"][0].data_ptr()
            else:                        # no optimizer for this arch: gradients to scratch
                a.ln_dgamma = lb["ln_pg"].data_ptr()
                a.ln_dbeta = lb["ln_pg"].data_ptr() + 4 * H
        return a

    def rec_forms(self):
        """{arch.layer: form} — which implementation each recurrent layer's time loops take:
        "persistent" (pkc_rnn_persist.hip, one launch per loop), "persistent grid-synchronised"
        (pkc_rnn_lstm_persist.hip), "bf16 steps" / "fp32 steps" (one launch per time step, bf16 or
        exact-fp32 step products), with "block-sparse U" (kmap tables) and "exact quantised-h" (QX)
        qualifiers; a BPTT that takes another form than its forward is named after a "/".  A cfg
        that falls back from the persistent loops (a fragment plan too long, H > 576, ...) shows it
        here (pkc_rnn_persist_form: the library's own decision for these arguments)."""
        names = {1: "persistent", 2: "persistent grid-synchronised"}
        out = {}
        for n in self.nodes:
            if not n.rec:
                continue
            for li in range(len(n.layers)):
                a = self._rnn_args(n, li, True, self.max_len)
                lb = n.lbuf[li]
                ff = L.lib().pkc_rnn_persist_form(C.byref(a), 0)
                fb = L.lib().pkc_rnn_persist_form(C.byref(a), 1)
                step = "bf16 steps" if a.step_bf16 else "fp32 steps"
                f = names.get(ff, step)
                if fb != ff:
                    f += " / BPTT " + names.get(fb, step)
                if not ff and lb.get("kmap_fwd") is not None:
                    f += ", block-sparse U"
                if a.qh_exact:
                    f += ", exact quantised-h"
                out["%s.%d" % (n.arch, li)] = f
        return out

    def _rec_inputs(self, n, li):
        """[(ptr, ld)] per gate of layer li's GEMM input, and the dW operand (final version)."""
        M, G = self.M, n.G
        sp, lb = n.layers[li], n.lbuf[li]
        if li == 0:
            vs = [self._version(n, n.qv0 + (g + 1 if n.reads else 0)) for g in range(G)]
            fin = self._final_version(n) if self.qsrc[n.qkey]["Q"] else self._src(n)
            return vs, fin
        prev = n.lbuf[li - 1]
        if not sp["ibits"]:
            v = (prev["y"].data_ptr(), prev["D"])
            return [v] * G, v
        K = lb["K"]
        vs = [(lb["xq"].data_ptr() + 4 * g * M * K, K) for g in range(G)]
        return vs, vs[-1]

    def _rec_fwd(self, n, s, train):
        M, T = self.M, self.T
        self._quant_chain(n, s)
        for li, (sp, lb) in enumerate(zip(n.layers, n.lbuf)):
            H, K = lb["H"], lb["K"]
            if li > 0 and sp["ibits"]:
                prev = n.lbuf[li - 1]
                self._k("fakequant_input x%d" % n.G, 0, 4.0 * M * K * (n.G + 2),
                        "pkc_fakequant_input", ptr(prev["y"]), ptr(lb["xq"]), M * K, sp["ibits"],
                        n.G, ptr(lb["qwork"]), s)
            xin, _ = self._rec_inputs(n, li)
            for g in range(n.G):
                x_ptr, ldx = xin[g]
                kt = self._wt(sp["W"][g], False)
                if kt is not None:            # block-sparse W: one problem, k-tile lists
                    sf = 1
                    pr = L.GemmProblem(a_kcontig=1, b_kcontig=1, M=M, N=H, K=K, splits=1, A=x_ptr,
                                       lda=ldx, B=n.wq(li, "W", g).data_ptr(), ldb=K,
                                       C=lb["zslab"].data_ptr(), ldc=H, slab_stride=M * H,
                                       ktiles=kt[0].data_ptr(), kmax=kt[1])
                    self._k("rnn_gemm_W %dx%dx%d sparse %.2f" % (M, H, K, kt[2]),
                            2.0 * M * H * K * kt[2], 4.0 * (M * K + H * K * kt[2] + M * H),
                            "pkc_gemm_grouped", self.prec, C.byref(pr), 1, s)
                else:
                    sf = _splits(M, H, K, MAX_SPLITS)
                    self._k("rnn_gemm_W %dx%dx%d" % (M, H, K), 2.0 * M * H * K,
                            4.0 * (M * K + H * K + sf * M * H), "pkc_gemm", self.prec, 1, 1, M, H, K,
                            C.c_void_p(x_ptr), ldx, ptr(n.wq(li, "W", g)), K, ptr(lb["zslab"]), H,
                            sf, M * H, s)
                bn = sp["bnm"][g]
                a = L.DenseFwdArgs(
                    M=M, N=H, nslab=sf, zslab=lb["zslab"].data_ptr(), slab_stride=M * H,
                    bias=sp["b"][g].data_ptr() if sp["b"][g] is not None else None,
                    norm=(L.NORM_BN_TRAIN if train else L.NORM_BN_EVAL) if sp["bn"] else L.NORM_NONE,
                    gamma=bn.weight.data_ptr(), beta=bn.bias.data_ptr(),
                    running_mean=bn.running_mean.data_ptr(), running_var=bn.running_var.data_ptr(),
                    momentum=0.05, eps=1e-5, save_mean=lb["sm"].data_ptr() + 4 * g * H,
                    save_invstd=lb["si"].data_ptr() + 4 * g * H, act=L.ACT["linear"], drop_p=0.0,
                    seed=0, step_ctr=None, stream_id=0, keep_in=None, keep_out=None,
                    xhat=lb["xhat"].data_ptr() + 4 * g * M * H,
                    out=lb["wpre"].data_ptr() + 4 * g * M * H,
                    count_n=M * (2 if sp["bidir"] else 1))
                self._k("rnn_bn_fwd H=%d" % H, 0, 4.0 * M * H * (sf + 2), "pkc_dense_fwd",
                        C.byref(a), ptr(lb["work"]), s)
            ra = self._rnn_args(n, li, train, T)
            if ra.step_bf16 or ra.qh_exact:   # this step's U (after the last update) as bf16
                for g in range(n.G):
                    self._k("cast_bf16 U", 0, 6.0 * H * H, "pkc_cast_bf16", ptr(n.wq(li, "U", g)),
                            C.c_void_p(ra.U_h[g]), H * H, s)
            self._k("rnn_fwd_loop T=%d H=%d" % (T, H), 2.0 * n.G * T * lb["B2"] * H * H,
                    4.0 * T * n.G * H * H, "pkc_rnn_fwd", C.byref(ra), s)
            self._loop_watch(ra, lb, False)

    def _forward_kernels(self, s, train, batch=None, defer_loss=False, pending=None):
        """pending: the previous step's deferred last launch (see _optim_kernels), run together
        with this step's gather."""
        slots = {}
        if pending and pending[0] == "fwd":
            slots = self._place_fwd_opt(pending[1])
            self._gemms([self._gather_op()] + slots.pop(None, []), s)
        elif pending:
            self._gemms([self._gather_op()] + list(pending), s)
        elif not self.external:
            self._gather(s, batch)
        if self.reg_terms and self.loss_heads:
            self._reg_loss_kernels(s)
        nodes, i = self.nodes, 0
        while i < len(nodes):
            n = nodes[i]
            if n.rec:
                self._rec_fwd(n, s, train)
                i += 1
                continue
            if n.W is None:
                self._fwd_epilogue(n, s, train)
                i += 1
                continue
            # output heads reading the same tensor (cd + mono senones) share one matmul launch
            grp = [n]
            while (n.head and i + len(grp) < len(nodes) and not nodes[i + len(grp)].rec
                   and nodes[i + len(grp)].head and nodes[i + len(grp)].src == n.src):
                grp.append(nodes[i + len(grp)])
            for g in grp:
                self._quant_chain(g, s)
            probs = [self._fwd_problem(g) for g in grp]
            if len(grp) == 1 and self._fused_fwd(n, probs[0], s, train, slots.get(n)):
                i += 1
                continue
            if len(grp) == 1 and train and self._colstats_fwd(n, probs[0], s):
                i += 1
                continue
            self._gemms(probs + slots.pop(n, []), s)
            if len(grp) > 1:
                self._nll_multi(grp, s, train)
            else:
                self._fwd_epilogue(n, s, train)
            i += len(grp)
        if self.loss_heads and not defer_loss:
            self._k("loss_finalize", 0, 4.0 * self.M * (self.n_loss_terms + 1),
                    "pkc_loss_finalize", self.n_loss_terms, ptr(self.loss_ptrs), ptr(self.loss_w),
                    self.M, ptr(self.err_layer.row_err), ptr(self.loss_out), ptr(self.loss_acc),
                    None if self.seq else ptr(self.ctr), s)

    def _loss_op(self):
        """The loss reduction (and batch-counter advance) as an operation of the first backward
        launch: it only needs the forward's per-row losses."""
        p = L.GemmProblem(kind=L.OP_LOSS, M=self.n_loss_terms, N=self.M,
                          A=self.loss_ptrs.data_ptr(), B=self.loss_w.data_ptr(),
                          C=self.loss_out.data_ptr(), X1=self.err_layer.row_err.data_ptr(),
                          X2=self.loss_acc.data_ptr(), X3=None if self.seq else self.ctr.data_ptr())
        return ("loss", 0.0, 4.0 * self.M * (self.n_loss_terms + 1), p)

    def _nll_multi(self, heads, s, train):
        """LogSoftmax/NLL of several heads in one launch."""
        args = (L.NllArgs * len(heads))()
        for i, n in enumerate(heads):
            self._fwd_epilogue(n, s, train, out=args[i])
        self._k("nll_multi[%s]" % ",".join(str(n.N) for n in heads), 0,
                sum(4.0 * self.M * n.N * (n.sf + 2) for n in heads), "pkc_nll_fused_multi", args,
                len(heads), s)

    # ------------------------------------------------------------------ backward
    def _grad_slabs(self, n):
        """(pointer, nslab) of dL/d(out of n) as the consumers' dX slabs, with their offsets.  The
        consumers share a budget of MAX_SPLITS slabs, or SLAB_BUDGET_MULTI (8) when several matmul
        layers read the output (the heads' shared input; the fused small-batch BN backward sums at
        most 8 in registers); the widest consumer gives up splits first."""
        M = self.M
        want = [1 if (c.W is None or self._wt(c.W, True) is not None)
                else _splits(M, c.K, c.N, c.sxcap) for c in n.consumers]
        budget = SLAB_BUDGET_MULTI if len(n.consumers) > 1 and not self.cap else MAX_SPLITS
        while sum(want) > budget and max(want) > 1:
            want[want.index(max(want))] -= 1
        off = 0
        n.cons_off = []
        for c, w in zip(n.consumers, want):
            c.sx = w
            n.cons_off.append(off)
            off += c.sx
        return off

    def _dense_bwd_pre(self, n, s):
        """dL/dz of a dense layer: the fused dropout / activation / BatchNorm backward over the
        consumers' dX slabs (a head's dlogits came from the forward; its bias gradient is an
        operation of the grouped backward launch, _bwd_problems)."""
        M = self.M
        # gradient of n's output: its consumers' dX slabs (an input norm consumer writes one), or
        # a recurrent node's layer-0 dX slabs when n is that node's input norm
        gs = getattr(n, "gsrc", None)
        if gs is not None:
            g_ptr, g_ns, g_st = gs[0].data_ptr(), gs[1], gs[2]
        else:
            g_ptr, g_ns, g_st = ((n.gslab.data_ptr(), n.sb, M * n.N) if n.gslab is not None
                                 else (None, 0, 0))
        if n.W is None and n.ln:             # input LayerNorm: gamma / beta and input gradients
            self._ln_bwd(n, s, C.c_void_p(g_ptr), g_ns, g_st, self._norm_dx(n), None)
            return
        if n.head:
            if n.ln:                         # dlogits are the LayerNorm output's gradient
                self._ln_bwd(n, s, ptr(n.dz_ln), 1, 0, n.dz, n.db)
            return
        a = L.DenseBwdArgs(M=M, N=n.N, nslab=g_ns, gslab=g_ptr,
                           slab_stride=g_st,
                           norm=L.NORM_BN_TRAIN if n.bn else L.NORM_NONE,
                           act=L.ACT[n.act], gamma=n.gamma.data_ptr(),
                           beta=n.beta.data_ptr(), save_invstd=n.save_invstd.data_ptr(),
                           xhat=n.xhat.data_ptr(),
                           keep=n.keep.data_ptr() if n.keep is not None else None,
                           drop_p=n.drop,
                           dz=(n.dz_ln if n.ln else self._norm_dx(n) if n.W is None else n.dz).data_ptr(),
                           dgamma=n.dgamma.data_ptr() if n.bn else None,
                           dbeta=n.dbeta.data_ptr() if n.bn else None,
                           dbias=n.db.data_ptr() if (n.b is not None and not n.ln) else None,
                           dz_bf16=n.dz_h.data_ptr() if (n.W is not None and n.dz_h is not None)
                           else None, dz_scratch=int(getattr(n, "dz_scratch", False)))
        if n.bn and getattr(n, "bn_sums", None) is not None:
            # SyncBN: local column sums (and local dgamma / dbeta), all-reduce, global apply
            self._k("dense_bwd_stats N=%d" % n.N, 0, 4.0 * M * n.N * (g_ns + 2), "pkc_dense_bwd_stats",
                    C.byref(a), ptr(n.work), ptr(n.bn_sums), s)
            self.sync_bn(n.bn_sums)
            self._k("dense_bwd_sync_apply N=%d" % n.N, 0, 4.0 * M * n.N * 3,
                    "pkc_dense_bwd_sync_apply", C.byref(a), ptr(n.work), ptr(n.bn_sums),
                    M * self.sync_bn.world, s)
        elif getattr(n, "bnb_now", False):   # statistics came with the consumer's dX matmul
            self._k("dense_bwd_pre N=%d" % n.N, 0, 4.0 * M * n.N * 3, "pkc_dense_bwd_pre",
                    C.byref(a), ptr(n.work), 128, s)
        else:
            self._k("dense_bwd N=%d" % n.N, 0, 4.0 * M * n.N * (g_ns + 3), "pkc_dense_bwd",
                    C.byref(a), ptr(n.work), s)
        if n.ln:
            # the Linear's bias sits in front of the LayerNorm (per-row statistics): its gradient
            # is the column sum of the LayerNorm's input gradient
            self._ln_bwd(n, s, ptr(n.dz_ln), 1, 0, n.dz, n.db)

    def _norm_dx(self, n):
        """Where an input normalisation writes its input gradient: its slab of the producer's
        gradient slabs (own dz when it reads a feature stream)."""
        if n.src[0] == "node" and n.src[1].gslab is not None:
            P = n.src[1]
            off = P.cons_off[P.consumers.index(n)]
            return P.gslab[off * self.M * P.N:(off + 1) * self.M * P.N]
        return n.dz

    def _ln_bwd(self, n, s, dy, nslab, stride, dx, dbias):
        M = self.M
        self._k("layernorm_bwd N=%d" % n.N, 0, 4.0 * M * n.N * (nslab + 4), "pkc_layernorm_bwd", M,
                n.N, nslab, dy, stride, ptr(n.ln_xhat), ptr(n.ln_gamma), ptr(n.ln_stat), ptr(dx),
                ptr(n.dgamma_ln), ptr(n.dbeta_ln), ptr(dbias), s)

    def _bwd_problems(self, n):
        """dW = dz^T X (into the flat gradient buffer) and, when the producer needs it,
        dX = dz W (into the producer's gradient slabs)."""
        M = self.M
        if n.W is None:
            return []
        a_ptr, lda = self._final_version(n) if self.qsrc[n.qkey]["Q"] else self._src(n)
        out = []
        if n.head and not n.ln:
            out.append(("db %d" % n.N, 0.0, 4.0 * M * n.N,
                        L.GemmProblem(kind=L.OP_COLSUM, M=M, N=n.N, A=n.dz.data_ptr(),
                                      C=n.db.data_ptr())))
        sdw = getattr(n, "sdw", 1)
        dzh = n.dz_h.data_ptr() if getattr(n, "dz_h", None) is not None else None
        pr = L.GemmProblem(a_kcontig=0, b_kcontig=0, M=n.N, N=n.K, K=M, splits=sdw,
                           A=n.dz.data_ptr(), lda=n.N, B=a_ptr, ldb=lda,
                           C=(n.dwslab if sdw > 1 else n.dW).data_ptr(), ldc=n.K,
                           slab_stride=n.N * n.K if sdw > 1 else 0)
        prh = self._h_variant(pr, dzh, None if self.qsrc[n.qkey]["Q"] else self._src_h(n))
        out += [("dW %dx%dx%d%s" % (n.N, n.K, M, " s%d" % sdw if sdw > 1 else ""),
                 2.0 * M * n.N * n.K, 4.0 * (M * n.N + M * n.K + sdw * n.N * n.K), pr,
                 None if prh is None else (2.0 * (M * n.N + M * n.K) + 4.0 * sdw * n.N * n.K, prh))]
        if n.src[0] == "fea" and self.want_dx:
            # external mode: dL/dx of the caller's input, one slab straight into ext_dx
            W = n.Wq if n.qbits else n.W
            pr = L.GemmProblem(a_kcontig=1, b_kcontig=0, M=M, N=n.K, K=n.N, splits=1,
                               A=n.dz.data_ptr(), lda=n.N, B=W.data_ptr(), ldb=n.K,
                               C=self.ext_dx.data_ptr() + 4 * n.src[1], ldc=self.F, slab_stride=0)
            kt = self._wt(n.W, True)
            if kt is not None:
                pr.ktiles, pr.kmax = kt[0].data_ptr(), kt[1]
            out.append(("dX %dx%dx%d ext" % (M, n.K, n.N), 2.0 * M * n.N * n.K,
                        4.0 * (M * n.N + n.N * n.K + M * n.K), pr))
        if n.src[0] == "node" and self.needs_grad[n.src[1]]:
            P = n.src[1]
            off = P.cons_off[P.consumers.index(n)]
            W = n.Wq if n.qbits else n.W
            pr = L.GemmProblem(a_kcontig=1, b_kcontig=0, M=M, N=n.K, K=n.N, splits=n.sx,
                               A=n.dz.data_ptr(), lda=n.N, B=W.data_ptr(), ldb=n.K,
                               C=P.gslab.data_ptr() + 4 * off * M * P.N, ldc=n.K,
                               slab_stride=M * n.K)
            kt, d = self._wt(n.W, True), 1.0
            if kt is not None:
                pr.ktiles, pr.kmax, d = kt[0].data_ptr(), kt[1], kt[2]
            prh = self._h_variant(pr, dzh, n.W_h.data_ptr() if n.W_h is not None else None)
            P.bnb_now = False
            if kt is None and self._bnb_ok(P, n, pr, prh):
                # P's BatchNorm-backward statistics in this dX matmul's epilogue: it writes
                # dy into P.dz and the column sums into P.work (_dense_bwd_pre finishes)
                for q in (pr, prh):
                    if q is not None:
                        q.C, q.X1 = P.dz.data_ptr(), C.addressof(P.bnb_epi)
                P.bnb_now = True
            out.append(("dX %dx%dx%d%s" % (M, n.K, n.N, " sparse %.2f" % d if kt is not None else ""),
                        2.0 * M * n.N * n.K * d, 4.0 * (M * n.N + n.N * n.K * d + n.sx * M * n.K),
                        pr, None if prh is None else
                        (2.0 * (M * n.N + n.N * n.K * d) + 4.0 * n.sx * M * n.K, prh)))
        return out

    def _bnb_ok(self, P, n, pr, prh):
        """Whether producer P's BatchNorm backward can take its statistics from the epilogue of
        consumer n's dX matmul pr (and its bf16 form prh): one consumer, one slab, training BN
        without LayerNorm / SyncBN, a large batch, the 128x128 body for both operand forms."""
        if not (BN_BWD_EPI and self.M > 128 and not self.seq and P.bn and not P.ln and not P.head
                and P.W is not None and len(P.consumers) == 1 and pr.splits == 1
                and getattr(P, "bn_sums", None) is None and (P.drop == 0 or P.keep is not None)):
            return False
        lib = L.lib()
        for prec, q in ((self.prec, pr), (L.PREC_BF16IN, prh)):
            if q is not None and lib.pkc_gemm_bnbwd_ok(prec, 1, 0, q.M, q.N, q.K, C.c_void_p(q.A),
                                                       q.lda, C.c_void_p(q.B), q.ldb) != 128:
                return False
        if getattr(P, "bnb_epi", None) is None:
            P.bnb_epi = L.BnBwdEpi(xhat=P.xhat.data_ptr(),
                                   keep=P.keep.data_ptr() if P.keep is not None else None,
                                   gamma=P.gamma.data_ptr(), beta=P.beta.data_ptr(),
                                   part=P.work.data_ptr(), act=L.ACT[P.act], drop_p=P.drop)
        return True

    def _dw_sum_op(self, n):
        """The slab sum of a split-K dW into the gradient (an operation of the next launch)."""
        return ("dW slab-sum %s x%d" % (n.name, n.sdw), 0.0, 4.0 * n.N * n.K * (n.sdw + 1),
                L.GemmProblem(kind=L.OP_SLABSUM, M=n.sdw, N=n.N * n.K, A=n.dwslab.data_ptr(),
                              C=n.dW.data_ptr(), slab_stride=n.N * n.K))

    def _dense_bwd(self, n, s):
        self._dense_bwd_pre(n, s)
        self._gemms(self._bwd_problems(n), s)

    def _rec_bwd(self, n, s, want_dx0=False, on_layer=None):
        """BPTT of a recurrent node, top layer first; on_layer(li) after layer li's weight
        gradients are queued (the data-parallel bucket cut)."""
        M, T = self.M, self.T
        gs = getattr(n, "gsrc", None)
        if gs is not None:                   # external mode: the caller's output gradient
            dy_t, dy_ns, dy_stride = gs[0], gs[1], gs[2]
        else:
            dy_t, dy_ns = n.gslab, n.sb
            dy_stride = M * n.N
        dy_ptr = dy_t.data_ptr()
        # tests: where each layer's dL/dy slabs sit (tests/test_gpu_steps.py re-reads them)
        trace = getattr(self, "rec_dy_trace", None)
        for li in reversed(range(len(n.layers))):
            sp, lb = n.layers[li], n.lbuf[li]
            H, K = lb["H"], lb["K"]
            if trace is not None:
                trace[(n.arch, li)] = (dy_t, dy_ns, dy_stride)
            ra = self._rnn_args(n, li, True, T)
            if dy_ns > 1 and n.dysum is not None:
                self._rec_slab_sum_ptr(dy_ptr, dy_ns, M * lb["D"], dy_stride, n.dysum, s)
                dy_ptr, dy_ns, dy_stride = n.dysum.data_ptr(), 1, M * lb["D"]
            ra.dy, ra.dy_nslab, ra.dy_slab_stride = dy_ptr, dy_ns, dy_stride
            self._k("rnn_bwd_loop T=%d H=%d" % (T, H), 2.0 * n.G * T * lb["B2"] * H * H,
                    4.0 * T * n.G * H * H, "pkc_rnn_bwd", C.byref(ra), ptr(lb["dpre"]), s)
            self._loop_watch(ra, lb, True)
            _, (x_ptr, ldx) = self._rec_inputs(n, li)
            hsrc = lb["hq"] if sp["ibits"] else lb["hs"]
            # bf16 step mode: the weight gradients read bf16 operand copies (BF16IN: half the
            # bytes each CU ingests) — dz_g written by the BatchNorm backward, dgates / h_{t-1}
            # by the bf16 step kernels, the layer input cast once here
            wbf = (bool(ra.step_bf16) and lb.get("dz_h") is not None and ldx == K
                   and n.cand is None)
            dzs = []
            for g in range(n.G):
                bn = sp["bnm"][g]
                a = L.DenseBwdArgs(M=M, N=H, nslab=1, gslab=lb["dpre"].data_ptr() + 4 * g * M * H,
                                   slab_stride=0, norm=L.NORM_BN_TRAIN if sp["bn"] else L.NORM_NONE,
                                   act=L.ACT["linear"], gamma=bn.weight.data_ptr(),
                                   beta=bn.bias.data_ptr(),
                                   save_invstd=lb["si"].data_ptr() + 4 * g * H,
                                   xhat=lb["xhat"].data_ptr() + 4 * g * M * H, keep=None, drop_p=0.0,
                                   dz=lb["dz"].data_ptr() + 4 * g * M * H,
                                   dgamma=lb["dgamma"][g].data_ptr() if sp["bn"] else None,
                                   dbeta=lb["dbeta"][g].data_ptr() if sp["bn"] else None,
                                   dbias=lb["db"][g].data_ptr() if lb["db"][g] is not None else None,
                                   dz_bf16=lb["dz_h"].data_ptr() + 2 * g * M * H if wbf else None)
                self._k("rnn_bn_bwd H=%d" % H, 0, 4.0 * M * H * 4, "pkc_dense_bwd", C.byref(a),
                        ptr(lb["work"]), s)
                dzs.append(lb["dz"].data_ptr() + 4 * g * M * H)
            h16 = None
            if wbf:
                self._k("rnn_cast_x_bf16 %dx%d" % (M, K), 0, 6.0 * M * K, "pkc_cast_bf16",
                        C.c_void_p(x_ptr), ptr(lb["xw_h"]), M * K, s)
                h16 = ([lb["dz_h"].data_ptr() + 2 * g * M * H for g in range(n.G)],
                       lb["xw_h"].data_ptr(), lb["hs_h"].data_ptr(), lb["dgates_h"].data_ptr())
            sums = self._rec_wgrads(n, lb, dzs, x_ptr, ldx, hsrc, s, h16)
            # dX = sum_g dz_g W_g (one slab group per gate) in one grouped launch, with the weight
            # gradients' slab sums riding along
            dxp, nx = [], 0
            if li > 0 or want_dx0:
                for g in range(n.G):
                    dz = dzs[g]
                    kt = self._wt(sp["W"][g], True)
                    if kt is not None:        # block-sparse W^T: one slab per gate
                        sx = 1
                        pr = L.GemmProblem(a_kcontig=1, b_kcontig=0, M=M, N=K, K=H, splits=1,
                                           A=dz, lda=H, B=n.wq(li, "W", g).data_ptr(), ldb=K,
                                           C=lb["dx"].data_ptr() + 4 * nx * M * K, ldc=K,
                                           slab_stride=M * K, ktiles=kt[0].data_ptr(), kmax=kt[1])
                        dxp.append(("dX%d %dx%dx%d sparse %.2f" % (g, M, K, H, kt[2]),
                                    2.0 * M * H * K * kt[2], 4.0 * (M * H + H * K * kt[2] + M * K), pr))
                    else:
                        sx = _splits(M, K, H, MAX_SPLITS)
                        pr = L.GemmProblem(a_kcontig=1, b_kcontig=0, M=M, N=K, K=H, splits=sx,
                                           A=dz, lda=H, B=n.wq(li, "W", g).data_ptr(), ldb=K,
                                           C=lb["dx"].data_ptr() + 4 * nx * M * K, ldc=K,
                                           slab_stride=M * K)
                        dxp.append(("dX%d %dx%dx%d" % (g, M, K, H), 2.0 * M * H * K,
                                    4.0 * (M * H + H * K + sx * M * K), pr))
                    nx += sx
            if dxp or sums:
                self._gemms(dxp + sums, s)
            if on_layer is not None:
                on_layer(li)
            dy_t, dy_ns, dy_stride = lb["dx"], nx, M * K
            dy_ptr = dy_t.data_ptr()
            if li == 0 and n.src[0] == "node":
                n.src[1].gsrc = (lb["dx"], nx, M * K)   # input norm: gradient = these dX slabs
            elif li == 0 and self.want_dx:           # external mode: dL/dx of the caller's input
                self._rec_slab_sum_ptr(lb["dx"].data_ptr(), nx, M * K, M * K, self.ext_dx, s)

    def _rec_wgrads(self, n, lb, dzs, x_ptr, ldx, hsrc, s, h16=None):
        """Every gate's dW_g = dz_g^T x (H x K over the M rows) and dU_g = dgates_g^T h_{t-1} (H x H
        over the T*B2 rows; GRU-type candidates: (r|z)*h_{t-1}) of one layer in ONE grouped launch.
        Both operands are m-contiguous; with bf16 products the launch's problems take the 128x128
        body (pkc_gemm_grouped_tile), whose tiles halve the bytes each CU ingests per flop against
        the 64x64 body.  The contraction is split (slabs into n.rslab) only when the launch has fewer
        than REC_WG_TARGET workgroups; returns the slab-sum operations for the next launch.
        h16: (dz_g copies, x copy, h copy, dgates copy) bf16 operand pointers (BF16IN form)."""
        H, K, M, T = lb["H"], lb["K"], self.M, self.T
        R2 = T * lb["B2"]
        lib = L.lib()
        probs = []
        for g in range(n.G):
            usrc = lb["rh"] if g == n.cand else hsrc
            hw = hu = None
            if h16 is not None:
                hw = (h16[0][g], H, h16[1], K)
                hu = (h16[3] + 2 * g * R2 * H, H, h16[2], H)
            probs.append(("dW%d" % g, H, K, M, dzs[g], H, x_ptr, ldx, lb["dW"][g], hw))
            probs.append(("dU%d" % g, H, H, R2, lb["dgates"].data_ptr() + 4 * g * R2 * H, H,
                          usrc.data_ptr(), H, lb["dU"][g], hu))
        prec = L.PREC_BF16IN if h16 is not None else self.prec
        tiles = 0
        for (_, Mq, Nq, Kq, A, lda, B, ldb, _, hq) in probs:
            if hq is not None:
                A, lda, B, ldb = hq
            te = lib.pkc_gemm_grouped_tile(prec, 0, 0, Mq, Nq, Kq, C.c_void_p(A), lda,
                                           C.c_void_p(B), ldb)
            tiles += -(-Mq // te) * -(-Nq // te)
        split = max(1, min(REC_DW_SPLITS, -(-REC_WG_TARGET // max(1, tiles))))
        gem, sums, off = [], [], 0
        for (lab, Mq, Nq, Kq, A, lda, B, ldb, out, hq) in probs:
            ss = max(1, min(split, Kq // 256))           # >= 256 rows of contraction per slab
            dst = n.rslab.data_ptr() + 4 * off if ss > 1 else out.data_ptr()
            pr = L.GemmProblem(a_kcontig=0, b_kcontig=0, M=Mq, N=Nq, K=Kq, splits=ss, A=A,
                               lda=lda, B=B, ldb=ldb, C=dst, ldc=Nq,
                               slab_stride=Mq * Nq if ss > 1 else 0)
            q = ("%s %dx%dx%d%s" % (lab, Mq, Nq, Kq, " s%d" % ss if ss > 1 else ""),
                 2.0 * Mq * Nq * Kq, 4.0 * (Mq * Kq + Nq * Kq + ss * Mq * Nq), pr)
            if hq is not None:
                ph = L.GemmProblem.from_buffer_copy(pr)
                ph.A, ph.lda, ph.B, ph.ldb = hq
                q = q + ((2.0 * (Mq * Kq + Nq * Kq) + 4.0 * ss * Mq * Nq, ph),)
            gem.append(q)
            if ss > 1:
                sums.append(("rnn slab-sum %s x%d" % (lab, ss), 0.0, 4.0 * Mq * Nq * (ss + 1),
                             L.GemmProblem(kind=L.OP_SLABSUM, M=ss, N=Mq * Nq, A=dst,
                                           C=out.data_ptr(), slab_stride=Mq * Nq)))
                off += ss * Mq * Nq
        self._gemms(gem, s)
        return sums

    def _rec_slab_sum(self, slab, ns, numel, out, s):
        """out = sum of ns split-K slabs of a recurrent weight gradient (one grouped launch)."""
        self._rec_slab_sum_ptr(slab.data_ptr(), ns, numel, numel, out, s)

    def _rec_slab_sum_ptr(self, a_ptr, ns, numel, stride, out, s):
        self._gemms([("rnn slab-sum x%d" % ns, 0.0, 4.0 * numel * (ns + 1),
                      L.GemmProblem(kind=L.OP_SLABSUM, M=ns, N=numel, A=a_ptr,
                                    C=out.data_ptr(), slab_stride=stride))], s)

    def _opt_op(self, n, parts=1):
        """The optimizer update of node n's parameters as operations of grouped launches: `parts`
        consecutive slices of its work-item list (int32 pairs), one per launch."""
        if n not in self.node_opt:
            return []
        nch, cmap, idx = self.node_opt[n]
        nparam = sum(self.opt_entries[i]["p"].numel() for i in idx)
        nbout = sum(self.opt_entries[i]["p"].numel() for i in idx
                    if self.opt_entries[i].get("bout") is not None)
        parts = max(1, min(parts, nch))
        ops, b = [], 0
        for k in range(parts):
            e = (nch * (k + 1)) // parts
            segs = self._opt_segs(cmap, b, e)
            ops.append(("opt %s%s" % (n.name, "" if parts == 1 else " [%d/%d]" % (k + 1, parts)), 0.0,
                        (20.0 * nparam + 2.0 * nbout) * (e - b) / nch,
                        L.GemmProblem(kind=L.OP_OPTIM, M=e - b, A=self.opt_desc.data_ptr(),
                                      B=cmap.data_ptr() + 8 * b,
                                      X1=C.addressof(segs) if segs is not None else None,
                                      N=len(segs) if segs is not None else 0)))
            b = e
        return ops

    def _bucket_cut(self):
        """Data parallelism: the node after whose dW launch the gradients of it and every later
        node (the tail of gflat: heads and top layers, finished first in the reverse pass) form
        the first all-reduce bucket — about a third of the buffer or more — so that collective
        overlaps the rest of the backward.  Returns (node, gflat offset) or (None, 0)."""
        if not hasattr(self, "_cut"):
            self._cut, self._cut_layer = (None, 0), None
            total = self.gflat.numel()
            for n in reversed(self.nodes):
                if not self.needs_grad[n] or n not in self.grad_off:
                    continue
                if n.rec:
                    # a recurrent node's gradients are laid out layer by layer (RecNode.params) and
                    # finish top layer first: the cut is after layer li's weight gradients
                    starts, off = {}, self.grad_off[n]
                    for p, key, _m in n.params():
                        starts.setdefault(key[1], off)
                        off += p.numel()
                    for li in sorted(starts, reverse=True):
                        if total - starts[li] >= total // 3 and starts[li] > 0:
                            self._cut, self._cut_layer = (n, starts[li]), li
                            break
                    if self._cut[0] is not None:
                        break
                    continue
                off = self.grad_off[n]
                if total - off >= total // 3 and off > 0:
                    self._cut = (n, off)
                    break
        return self._cut

    def _backward_kernels(self, s, loss_op=None, spread_opt=False, on_cut=None, fwd_defer=False):
        """Reverse pass.  The matmuls of a layer (dW, dX) are queued and launched together with
        those of the layers after it that are still pending, right before the first kernel that
        needs one of their results (the producer's BatchNorm backward reads the dX slabs).
        spread_opt: each layer's optimizer update joins the launch AFTER the one holding its dW
        and dX (dX still reads the old weights), so the bandwidth-bound update overlaps the
        latency-bound matmuls instead of running as its own launch at the end.  An update of more
        than OPT_SPREAD_PARAMS parameters is cut into parts over the following launches, so no
        single launch carries a whole output head's update."""
        spread_opt = spread_opt and not self.reg_terms
        for n in self.nodes:
            if n.gslab is not None:
                n.sb = self._grad_slabs(n)
        pend = [loss_op] if loss_op is not None else []
        self.fwd_opt = []       # fwd_defer: (node, update op) for the next step's forward
        future = [[], []]       # future[i]: operations riding in the i-th launch from now
        cut_node = self._bucket_cut()[0] if on_cut is not None else None
        cut_wait = -1           # launches until the cut node's gradient is final
        pend_nodes = []

        def flush():
            nonlocal pend, future, pend_nodes, cut_node, cut_wait
            now = future.pop(0)
            if pend or now:
                self._gemms(pend + now, s)
            pend = []
            while len(future) < 2:
                future.append([])
            if cut_wait > 0:
                cut_wait -= 1
            if cut_node is not None and cut_node in pend_nodes:
                # a split-K dW becomes final one launch later (its slab sum).  Output heads do not
                # flush, so sibling heads can share the cut node's launch: wait for the slowest of
                # them (an unsplit cut head beside a split one would otherwise ship the split
                # head's stale dW in the first bucket)
                cut_wait = 1 if any(getattr(p, "sdw", 1) > 1 for p in pend_nodes) else 0
                cut_node = None
            if cut_wait == 0:
                cut_wait = -1
                on_cut()                # the first bucket's gradients are final
            pend_nodes = []

        for n in reversed(self.nodes):
            if not self.needs_grad[n]:
                continue
            if n.rec:
                flush()
                on_layer = None
                if cut_node is n:               # sequence DP: first bucket after a layer's grads
                    cut_node = None
                    on_layer = (lambda li: on_cut() if li == self._cut_layer else None)
                self._rec_bwd(n, s, want_dx0=n.src[0] == "node" or self.want_dx, on_layer=on_layer)
                continue
            if not n.head:
                flush()
            self._dense_bwd_pre(n, s)
            pend += self._bwd_problems(n)
            pend_nodes.append(n)
            lag = 1
            if getattr(n, "sdw", 1) > 1 and n.W is not None:
                future[1].append(self._dw_sum_op(n))    # the launch after the dW's
                lag = 2                                 # its update one launch later still
            if spread_opt:
                nparam = sum(self.opt_entries[i]["p"].numel() for i in self.node_opt.get(n, (0, 0, []))[2])
                parts = -(-nparam // OPT_SPREAD_PARAMS) if OPT_SPREAD_PARAMS > 0 else 1
                if fwd_defer:                   # the next step's forward launches carry them
                    self.fwd_opt += [(n, op) for op in self._opt_op(n, parts)]
                    continue
                for k, op in enumerate(self._opt_op(n, parts)):
                    while len(future) <= lag + k:
                        future.append([])
                    future[lag + k].append(op)
        flush()
        # operations still to run, merged into as few launches as the order allows (a layer's
        # update never shares a launch with the slab sum of its own gradient)
        self.spread_tail = []
        cur, summed = [], set()
        for f in future:
            if any(op[0].startswith("opt ") and op[0][4:].split(" ")[0] in summed for op in f):
                self.spread_tail.append(cur)
                cur, summed = [], set()
            cur = cur + f
            summed |= {op[0].split(" ")[2] for op in f if op[0].startswith("dW slab-sum ")}
        if cur:
            self.spread_tail.append(cur)
        if not spread_opt:
            for f in self.spread_tail:       # slab sums, before the all-reduce / optimizer
                self._gemms(f, s)
            self.spread_tail = []
            if cut_wait >= 0:
                on_cut()

    def _build_reg(self):
        """Device descriptors of the regulariser terms (item lists, block starts, buffers)."""
        grads = {id(e["p"]): e["g"] for e in self.opt_entries}
        only = {id(e["p"]) for e in self.opt_entries if e.get("reg_only")}
        for t in self.reg_terms:
            items, bstart = t.items(grads)
            arr = (L.RegItem * len(items))()
            for i, (p, g, ld, r0, r1, c0, c1, blk) in enumerate(items):
                arr[i] = L.RegItem(p=p.data_ptr(), g=None if g is None else g.data_ptr(), ld=ld,
                                   r0=r0, r1=r1, c0=c0, c1=c1, block=blk,
                                   assign=1 if id(p) in only else 0)
            t.nitems, t.nblocks = len(items), len(bstart) - 1
            t.items_dev = torch.frombuffer(bytearray(C.string_at(arr, C.sizeof(arr))),
                                           dtype=torch.uint8).to(self.dev)
            t.bstart = torch.tensor(bstart, dtype=torch.int32, device=self.dev)
            t.partial = _f32(len(items), self.dev)
            t.coef = _f32(t.nblocks, self.dev)
            t.nparam = sum(p.numel() for p in t.params)

    def _reg_loss_kernels(self, s):
        """Regulariser values of the current weights (before the forward's loss reduction)."""
        for t in self.reg_terms:
            self._k("reg_partial", 0, 4.0 * t.nparam, "pkc_reg_partial", t.kind, ptr(t.items_dev),
                    t.nitems, ptr(t.partial), s)
            self._k("reg_finalize", 0, 4.0 * (t.nitems + self.Mmax), "pkc_reg_finalize", t.kind,
                    ptr(t.bstart), t.nblocks, ptr(t.partial), C.c_float(t.lam), ptr(t.coef),
                    ptr(t.row_loss), self.Mmax, s)

    def _reg_grad_kernels(self, s):
        """d(w * lam * norms)/dp added to the (all-reduced) gradients before the optimizer."""
        for t in self.reg_terms:
            if t.loss_weight != 1.0:
                raise NotImplementedError("a weighted regulariser term in loss_final")
            self._k("reg_grad", 0, 12.0 * t.nparam, "pkc_reg_grad", t.kind, ptr(t.items_dev),
                    t.nitems, ptr(t.coef), s)

    def _optim_kernels(self, s, spread_opt=False, defer=False):
        """defer (spread mode): when the step's last launch holds weight updates only, return its
        operations instead of launching them — the next step's first launch (its batch gather,
        which reads neither) carries them (multi-step graphs; the graph's last step flushes)."""
        if not self.opt_entries:
            return None
        spread_opt = spread_opt and not self.reg_terms
        self._reg_grad_kernels(s)
        if spread_opt:
            if getattr(self, "fwd_opt", None):
                # fwd_defer: every update waits for the next step's forward (_place_fwd_opt)
                for f in self.spread_tail:
                    self._gemms(f, s)
                pend, self.fwd_opt = ("fwd", self.fwd_opt), []
                return pend
            tail, pend = self.spread_tail, None
            if (defer and DEFER_TAIL and tail and not self.prune_list and not self.seq
                    and self.loss_heads and len(tail[-1]) < 8
                    and all(op[3].kind == L.OP_OPTIM for op in tail[-1])):
                tail, pend = tail[:-1], tail[-1]
            for f in tail:
                self._gemms(f, s)
            if pend is None:
                self._prune_kernels(s)
            return pend
        nparam = sum(e["p"].numel() for e in self.opt_entries)
        self._k("optim_step", 0, 4.0 * nparam * 5, "pkc_optim_step", ptr(self.opt_desc),
                len(self.opt_entries), ptr(self.opt_map), self.opt_nchunks, s)
        self._prune_kernels(s)

    def _train_step_kernels(self, allreduce=None, batch=None):
        s = self._stream()
        defer = bool(self.loss_heads)
        spread = not self.seq and allreduce is None
        self._forward_kernels(s, True, batch, defer_loss=defer)
        works = []
        cut_off = self._bucket_cut()[1] if allreduce is not None else 0

        def first_bucket():             # overlaps the rest of the backward
            works.append(allreduce(self.gflat[cut_off:], async_op=True))

        self._backward_kernels(s, self._loss_op() if defer else None, spread_opt=spread,
                               on_cut=first_bucket if (allreduce is not None and cut_off) else None)
        if allreduce is not None:
            if works:
                works.append(allreduce(self.gflat[:cut_off], async_op=True))
            else:
                works.append(allreduce(self.gflat, async_op=True))
            for w in works:
                if w is not None:
                    w.wait()
        self._optim_kernels(s, spread_opt=spread)

    # ------------------------------------------------------------------ public API
    def _set_rows(self, batch):
        if self.seq:
            self.T = batch[3]
            self.M = self.T * self.B
        else:
            self.M = self.B

    def train_step(self, allreduce=None, batch=None):
        """One batch: forward, backward, [allreduce(flat grads)], optimizer (core.py:216-232).
        Sequence models: batch = next_seq_batch() (drawn here when None)."""
        if self.seq:
            batch = batch or self.next_seq_batch()
            self._set_rows(batch)
            if self.frame_scales is not None:
                # sequence DP: rank r's padded batch has T_r * B rows; scale its mean loss by its
                # share of all ranks' rows, so the summed gradient is that of the mean over every
                # row of the global batch, not the mean of unequal batch means
                self.grad_scale = float(self.frame_scales[getattr(batch, "index", self.batch_i)])
            self._upload_seq_meta(batch)
            if (self.seq_graphs is not None and allreduce is None and self.frame_scales is None
                    and self._seq_seen(batch)):
                self._seq_graph(batch).replay()
            else:
                self._train_step_kernels(allreduce, batch)
                self.ctr.add_(1)           # step counter of the dropout RNG streams
        elif self.graph is not None:
            if self.graph_opt is not None and self.graph_tail is not None:
                # bucketed: first bucket all-reduced while the rest of the backward replays
                self.graph.replay()
                off = self._bucket_cut()[1]
                works = [allreduce(self.gflat[off:], async_op=True)] if allreduce else []
                self.graph_tail.replay()
                if allreduce:
                    works.append(allreduce(self.gflat[:off], async_op=True))
                for w in works:
                    if w is not None:
                        w.wait()
                self.graph_opt.replay()
            else:
                self.graph.replay()
                if self.graph_opt is not None:
                    if allreduce is not None:
                        allreduce(self.gflat)
                    self.graph_opt.replay()
        else:
            self._set_rows(None)
            self._train_step_kernels(allreduce)
        self._after_step()

    def train_steps(self, n, allreduce=None):
        """n consecutive training batches (core.py:216-232 per batch); whole multi-step graphs
        where possible."""
        if self.graph is not None and self.graph_multi is not None and allreduce is None:
            k = self.steps_per_graph
            while n >= k:
                self.graph_multi.replay()
                for _ in range(k):
                    self._after_step()
                n -= k
        for _ in range(n):
            self.train_step(allreduce)

    def eval_step(self, batch=None):
        """Validation batch: forward with running BN statistics, loss/err accumulated."""
        if self.seq:
            batch = batch or self.next_seq_batch()
        self._set_rows(batch)
        if self.seq:
            self._upload_seq_meta(batch)
        self._forward_kernels(self._stream(), False, batch)

    def profile_step(self):
        """Run one eager training step with events around every launch; returns
        [(label, fn, flops, bytes, ms)] (device time per launch)."""
        self.prof = []
        self._set_rows(None)
        self._train_step_kernels()
        torch.cuda.synchronize()
        out = [(l, f, fl, nb, e0.elapsed_time(e1)) for (l, f, fl, nb, e0, e1, _) in self.prof]
        self.last_prof_calls = [(l, f, a) for (l, f, _, _, _, _, a) in self.prof]
        self.prof = None
        self._after_step()
        return out

    def step_cost_of(self, label, reps=50):
        """In-step device time (us) of the launches labelled `label`: the captured step graph
        timed with and without them (HIP events around `reps` replays each).  The launches are
        measured where they run — after their real producers, inside the step — so this agrees
        with rocprofv3's per-dispatch durations of the step graph.  Corrupts the training state
        (the skipped outputs go stale): call it after the timed region only."""
        def graph_us(skip):
            self.skip_labels = set(skip)
            self._set_rows(None)
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                s = self._stream()
                self._forward_kernels(s, True, defer_loss=bool(self.loss_heads))
                self._backward_kernels(s, self._loss_op() if self.loss_heads else None,
                                       spread_opt=True)
                self._optim_kernels(s, spread_opt=True)
            torch.cuda.current_stream().wait_stream(st)
            self.skip_labels = set()
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            best = None
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    g.replay()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / reps
                best = us if best is None else min(best, us)
            return best
        full = graph_us(())
        without = graph_us(tuple(label) if isinstance(label, (list, tuple, set)) else (label,))
        return full - without, full

    def replay_launches(self, fn, reps):
        """Re-issue every launch of entry point `fn` of the last profile_step, `reps` rounds
        (eager; for PMC counter runs — corrupts the training state)."""
        calls = [(f, a) for (l, f, a) in self.last_prof_calls if f == fn]
        for _ in range(reps):
            for f, a in calls:
                call(f, *a[:-1], self._stream())
        torch.cuda.synchronize()
        return len(calls)

    def _after_step(self):
        self.steps_done += 1
        for e in self.opt_entries:
            e["step"] += 1
        if self.opt_entries and not self.static_opt and self.graph is None:
            self._upload_opt_desc(step_inc=1)

    def _seq_seen(self, batch):
        """Whether this batch's padded length has a graph or has now been seen SEQ_CAPTURE_AFTER
        times (counted per chunk, with the graphs)."""
        T = int(batch[3])
        if T in self.seq_graphs:
            return True
        n = self.seq_seen.get(T, 0) + 1
        self.seq_seen[T] = n
        return n >= SEQ_CAPTURE_AFTER

    def _seq_graph(self, batch):
        """The captured training step of a sentence batch of padded length T (captured on first
        use, kept in an LRU of SEQ_GRAPHS): every launch of the step — gather, recurrent time
        loops, heads, backward, optimizer — and the dropout step counter's increment.  Its inputs
        are the device-side batch metadata (seq_meta, uploaded before the replay), the chunk and
        the device step counters, so one graph serves every batch of that T."""
        T = int(batch[3])
        g = self.seq_graphs.pop(T, None)
        if g is None:
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st, pool=self.seq_pool):
                self._train_step_kernels(None, batch)
                self.ctr.add_(1)
            torch.cuda.current_stream().wait_stream(st)
            self.seq_captures += 1
            while len(self.seq_graphs) >= max(1, SEQ_GRAPHS):
                self.seq_graphs.pop(next(iter(self.seq_graphs)))
        self.seq_graphs[T] = g                  # most recently used last
        return g

    def capture(self, split_optimizer=False, steps_per_graph=8):
        """Capture the training step into hipGraph(s) (models with step-independent optimizer
        descriptors: RMSprop / momentum-free SGD).  split_optimizer=True captures
        forward+backward and the optimizer separately so a gradient all-reduce fits in between.
        Without the split, a second graph holds steps_per_graph consecutive steps (the batch
        counter lives on the device), so train_steps() pays one graph launch per that many
        batches instead of one per batch.  Sequence models: per padded length T, each step's
        launches are captured the first time a batch of that T trains and replayed after that
        (single-process steps with a fixed loss scale; data-parallel steps stay eager)."""
        if self.seq:
            if not self.static_opt or self.sync_bn is not None or self.external:
                return False
            self.seq_graphs, self.seq_pool, self.seq_captures = {}, torch.cuda.graph_pool_handle(), 0
            self.seq_seen = {}
            return True
        if not self.static_opt or self.sync_bn is not None:
            return False             # SyncBN: collectives inside the forward / backward, eager
        self._set_rows(None)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())

        def one_step(st, pending=None, defer_tail=False):
            defer = bool(self.loss_heads)
            self._forward_kernels(st, True, defer_loss=defer, pending=pending)
            fwd = (OPT_FWD and defer_tail and not split_optimizer and not self.prune_list
                   and not self.reg_terms and self.M <= 128 and bool(self.loss_heads))
            self._backward_kernels(st, self._loss_op() if defer else None,
                                   spread_opt=not split_optimizer, fwd_defer=fwd)
            if not split_optimizer:
                return self._optim_kernels(st, spread_opt=True, defer=defer_tail)
            return None

        self.graph_tail = None
        if split_optimizer and self._bucket_cut()[0] is not None:
            # data parallelism: forward + backward up to the first bucket's last dW launch, then
            # the rest of the backward, as two graphs with the first all-reduce between them
            pool = torch.cuda.graph_pool_handle()
            g, gt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                g.capture_begin(pool=pool)

                def cut():
                    g.capture_end()
                    gt.capture_begin(pool=pool)

                st = self._stream()
                defer = bool(self.loss_heads)
                self._forward_kernels(st, True, defer_loss=defer)
                self._backward_kernels(st, self._loss_op() if defer else None, spread_opt=False,
                                       on_cut=cut)
                gt.capture_end()
            self.graph_tail = gt
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                one_step(self._stream())
        self.graph_multi, self.steps_per_graph = None, 1
        if not split_optimizer and steps_per_graph > 1:
            gm = torch.cuda.CUDAGraph()
            n0 = self.n_launches
            with torch.cuda.graph(gm, stream=s):
                pend = None
                for k in range(steps_per_graph):
                    pend = one_step(self._stream(), pend, defer_tail=k < steps_per_graph - 1)
            self.graph_launches_per_step = (self.n_launches - n0) / steps_per_graph
            self.graph_multi, self.steps_per_graph = gm, steps_per_graph
        self.graph_opt = None
        if split_optimizer:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, stream=s):
                self._optim_kernels(self._stream())
            self.graph_opt = g2
        torch.cuda.current_stream().wait_stream(s)
        self.graph = g
        return True

    def _loop_watch(self, ra, lb, bwd):
        """After a layer's pkc_rnn_fwd / pkc_rnn_bwd: when it ran as a grid-synchronised loop,
        add its timeout word (rwork[4 B2 H + 1], zeroed by the launch) to loop_fail."""
        key = (id(lb), bwd, ra.T)
        form = self._loop_forms.get(key)
        if form is None:
            form = self._loop_forms[key] = L.lib().pkc_rnn_persist_form(C.byref(ra), int(bwd))
        if form == 2 and not (bwd and ra.T < 2):
            o = 4 * lb["B2"] * lb["H"] + 1
            self.loop_fail.add_(lb["rwork"][o:o + 1].view(torch.int32))

    def _check_loops(self):
        if int(self.loop_fail.item()) != 0:
            raise L.PkcError("a grid-synchronised recurrent time loop gave up waiting for its peer "
                             "workgroups (%d launch(es)): the GPU was shared with another persistent "
                             "kernel or the grid was not co-resident; set PKC_RNN_LSTM_PERSIST=0 / "
                             "PKC_RNN_LIGRU_GRID=0 to use the per-step launches"
                             % int(self.loop_fail.item()))

    def loss_values(self):
        """(loss_final, err) of the last step (forces a sync)."""
        v = self.loss_out.cpu()
        self._check_loops()
        return float(v[0]), float(v[1])

    def chunk_totals(self):
        """(loss_sum, err_sum) over the batches since bind_chunk (core.py:251-252)."""
        v = self.loss_acc.cpu()
        self._check_loops()
        return float(v[0]), float(v[1])

    def head_output(self, out_name):
        """(M, N) view of a head / layer output of the current batch."""
        n = self.produced[out_name]
        return n.out[:self.M * n.N].view(self.M, n.N)

    def sync_state(self):
        """Reflect the step count into BN num_batches_tracked (nn.BatchNorm1d increments it on
        every training forward; the kernels update running stats but not this counter)."""
        for n in self.nodes:
            if n.rec:
                for sp in n.layers:
                    if sp["bn"]:
                        for g, bn in enumerate(sp["bnm"]):
                            bn.num_batches_tracked.fill_(sp["nbt0"][g] + self.steps_done)
            elif n.bn:
                n.spec["nbt"].fill_(n.nbt0 + self.steps_done)

    def optimizer_state_dict(self, arch):
        """torch.optim state_dict of one architecture's optimizer (core.py:317-322).

        param_groups come from the torch.optim class utils.optimizer_init would build
        (utils.py:1833-1881) over the same parameters, so every hyperparameter key of the running
        torch version is present and the dict loads into the reference's optimizer and steps."""
        net = self.nets[arch]
        params = list(net.parameters())
        index = {id(p): i for i, p in enumerate(params)}
        o = self.arch_opts[arch]
        kind = o["arch_opt"]
        state = {}
        for e in self.opt_entries:
            if e["arch"] != arch or (e["step"] == 0 and not e.get("has_buf")):
                continue
            if kind == "sgd":
                if float(o["opt_momentum"]) == 0:
                    continue                      # torch SGD keeps no state without momentum
                st = {"momentum_buffer": e["s1"].detach().cpu().clone()}
            elif kind == "rmsprop":
                st = {"step": torch.tensor(float(e["step"])),
                      "square_avg": e["s1"].detach().cpu().clone()}
                if e["s3"] is not None:
                    st["momentum_buffer"] = e["s3"].detach().cpu().clone()
                if e["s2"] is not None:
                    st["grad_avg"] = e["s2"].detach().cpu().clone()
            else:
                st = {"step": torch.tensor(float(e["step"])),
                      "exp_avg": e["s1"].detach().cpu().clone(),
                      "exp_avg_sq": e["s2"].detach().cpu().clone()}
                if e["s3"] is not None:
                    st["max_exp_avg_sq"] = e["s3"].detach().cpu().clone()
            state[index[id(e["p"])]] = st
        group = torch_optimizer(params, o).state_dict()["param_groups"][0]
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, arch, sd):
        """optimizers[net].load_state_dict(checkpoint['optimizer_par']) (core.py:114-121)."""
        net = self.nets[arch]
        params = list(net.parameters())
        index = {id(p): i for i, p in enumerate(params)}
        for e in self.opt_entries:
            if e["arch"] != arch:
                continue
            st = sd["state"].get(index[id(e["p"])])
            if not st:
                continue
            if "square_avg" in st:
                e["s1"].copy_(st["square_avg"])
            if "grad_avg" in st and e["s2"] is not None:
                e["s2"].copy_(st["grad_avg"])
            if "exp_avg" in st:
                e["s1"].copy_(st["exp_avg"])
                e["s2"].copy_(st["exp_avg_sq"])
            if "max_exp_avg_sq" in st and e["s3"] is not None:
                e["s3"].copy_(st["max_exp_avg_sq"])
            if st.get("momentum_buffer") is not None:
                (e["s3"] if e["s3"] is not None else e["s1"]).copy_(st["momentum_buffer"])
                e["has_buf"] = True       # torch SGD: a loaded buffer is continued, not reset
            if "step" in st:
                e["step"] = int(float(st["step"]))
        self._upload_opt_desc(step_inc=1)


def torch_optimizer(params, o):
    """The torch.optim object utils.optimizer_init (utils.py:1833-1881) builds for cfg section o."""
    lr = float(o["arch_lr"])
    kind = o["arch_opt"]
    if kind == "sgd":
        return torch.optim.SGD(params, lr=lr, momentum=float(o["opt_momentum"]),
                               weight_decay=float(o["opt_weight_decay"]),
                               dampening=float(o["opt_dampening"]),
                               nesterov=_b(o["opt_nesterov"]))
    if kind == "adam":
        return torch.optim.Adam(params, lr=lr, betas=[float(v) for v in o["opt_betas"].split(",")],
                                eps=float(o["opt_eps"]), weight_decay=float(o["opt_weight_decay"]),
                                amsgrad=_b(o["opt_amsgrad"]))
    if kind == "rmsprop":
        return torch.optim.RMSprop(params, lr=lr, momentum=float(o["opt_momentum"]),
                                   alpha=float(o["opt_alpha"]), eps=float(o["opt_eps"]),
                                   centered=_b(o["opt_centered"]),
                                   weight_decay=float(o["opt_weight_decay"]))
    raise NotImplementedError("arch_opt=%s" % kind)


class ModuleRunner:
    """Forward of one MLP module on the pkc kernels for any row count <= max_rows (MLP.forward for
    stand-alone calls, and the per-utterance forward of run_nn's forward mode)."""

    def __init__(self, net, max_rows, inp_dim):
        net.check_supported()
        self.net, self.rows, self.dev = net, max_rows, next(net.parameters()).device
        self.specs = net.layer_specs()
        self.norms = net.input_norm_specs() if hasattr(net, "input_norm_specs") else []
        self.nbufs = [dict(y=_f32(max_rows * inp_dim, self.dev), xh=_f32(max_rows * inp_dim, self.dev),
                           st=_f32(2 * max_rows, self.dev), sm=_f32(inp_dim, self.dev),
                           si=_f32(inp_dim, self.dev),
                           work=_f32(L.lib().pkc_dense_work_size(max_rows, inp_dim), self.dev))
                      for _ in self.norms]
        self.bufs = []
        K = inp_dim
        for sp in self.specs:
            N = sp["out"]
            b = dict(z=_f32(MAX_SPLITS * max_rows * N, self.dev), K=K, N=N,
                     xhat=_f32(max_rows * N, self.dev), sm=_f32(N, self.dev),
                     si=_f32(N, self.dev), out=_f32(max_rows * N, self.dev),
                     work=_f32(L.lib().pkc_dense_work_size(max_rows, N), self.dev))
            if sp["ln"]:
                b.update(ly=_f32(max_rows * N, self.dev), lxh=_f32(max_rows * N, self.dev),
                         lst=_f32(2 * max_rows, self.dev))
            if sp["quant"]:
                b["Wq"] = torch.zeros_like(sp["W"])
            if sp["inp_quant"]:
                b["xq"] = _f32(max_rows * K, self.dev)
                b["qwork"] = _f32(256, self.dev)
            self.bufs.append(b)
            K = N
        self.prune_work = None
        self.eff = pattern_effective_masks(net, Engine._stream())
        # the reference re-prunes / re-applies pattern^L on every forward call
        self.prunes = any(sp.get("prune") is not None for sp in self.specs) or bool(self.eff)
        if not self.prunes:          # else refreshed at the top of every run()
            self.refresh()

    def refresh(self):
        """Re-apply HCGS masks / the QuantizeLinear clamp and re-quantise (after weights change)."""
        s = Engine._stream()
        for sp, b in zip(self.specs, self.bufs):
            qb = int(sp["quant"] or 0)
            mask = self.eff.get(id(sp["W"]), sp["mask"])
            if sp.get("prune") is not None:      # mask, then prune (neural_networks.py:256-278)
                if mask is not None:
                    call("pkc_apply_mask", ptr(sp["W"]), ptr(mask), sp["W"].numel(),
                         C.c_float(0.0), s)
                if self.prune_work is None:
                    self.prune_work = torch.zeros(L.lib().pkc_prune_work_size(), dtype=torch.uint8,
                                                  device=self.dev)
                call("pkc_prune", ptr(sp["W"]), sp["W"].numel(), C.c_double(float(sp["prune"])), None,
                     ptr(self.prune_work), s)
                if qb:
                    call("pkc_apply_mask", ptr(sp["W"]), None, sp["W"].numel(), C.c_float(1.0), s)
            elif mask is not None or qb:
                call("pkc_apply_mask", ptr(sp["W"]), ptr(mask), sp["W"].numel(),
                     C.c_float(1.0 if qb else 0.0), s)
            if qb:
                call("pkc_fakequant_weight", ptr(sp["W"]), ptr(b["Wq"]), sp["W"].numel(), qb, s)

    def run(self, x_ptr, ld, M, train=False, log_prior=None):
        """x_ptr: device address of an (M, ld) fp32 matrix; returns the (M, N) output view.
        With input quantisation on the first layer, self.input_version holds the address of the
        quantised input (the value the reference leaves in the caller's tensor)."""
        assert M <= self.rows
        if self.prunes:
            self.refresh()
        s = Engine._stream()
        cur, cld = x_ptr, ld
        self.input_version = None
        for ns, nb in zip(self.norms, self.nbufs):       # input LayerNorm / BatchNorm
            K0 = self.bufs[0]["K"]
            if cld != K0:
                raise NotImplementedError("input normalisation of a strided feature stream")
            if ns["kind"] == "ln":
                call("pkc_layernorm_fwd", M, K0, 1, C.c_void_p(cur), 0, None, ptr(ns["gamma"]),
                     ptr(ns["beta"]), C.c_float(1e-6), ptr(nb["y"]), ptr(nb["xh"]), ptr(nb["st"]), s)
            else:
                a = L.DenseFwdArgs(
                    M=M, N=K0, nslab=1, zslab=cur, slab_stride=0, bias=None,
                    norm=L.NORM_BN_TRAIN if train else L.NORM_BN_EVAL, gamma=ns["gamma"].data_ptr(),
                    beta=ns["beta"].data_ptr(), running_mean=ns["rm"].data_ptr(),
                    running_var=ns["rv"].data_ptr(), momentum=0.05, eps=1e-5,
                    save_mean=nb["sm"].data_ptr(), save_invstd=nb["si"].data_ptr(), act=0,
                    xhat=nb["xh"].data_ptr(), out=nb["y"].data_ptr(), count_n=0)
                call("pkc_dense_fwd", C.byref(a), ptr(nb["work"]), s)
            cur = nb["y"].data_ptr()
        for li, (sp, b) in enumerate(zip(self.specs, self.bufs)):
            N, K = b["N"], b["K"]
            if sp["inp_quant"]:
                if cld != K:
                    raise NotImplementedError("input quantisation of a strided feature stream")
                call("pkc_fakequant_input", C.c_void_p(cur), ptr(b["xq"]), M * K,
                     int(sp["inp_quant"]), 1, ptr(b["qwork"]), s)
                cur = b["xq"].data_ptr()
                if li == 0:
                    self.input_version = cur
            W = b["Wq"] if sp["quant"] else sp["W"]
            sf = _splits(M, N, K, MAX_SPLITS)
            call("pkc_gemm", L.PREC_FP32, 1, 1, M, N, K, C.c_void_p(cur), cld, ptr(W), K,
                 ptr(b["z"]), N, sf, M * N, s)
            zp, zs, bias = b["z"].data_ptr(), M * N, sp["b"].data_ptr()
            if sp["ln"]:
                call("pkc_layernorm_fwd", M, N, sf, C.c_void_p(zp), zs, C.c_void_p(bias),
                     ptr(sp["ln_gamma"]), ptr(sp["ln_beta"]), C.c_float(1e-6), ptr(b["ly"]),
                     ptr(b["lxh"]), ptr(b["lst"]), s)
                zp, zs, bias, sf = b["ly"].data_ptr(), 0, None, 1
            if sp["act"] == "softmax":
                a = L.NllArgs(M=M, N=N, nslab=sf, zslab=zp, slab_stride=zs,
                              bias=bias, labels=None, label_stride=0, weight=0.0,
                              logp=b["out"].data_ptr(),
                              log_prior=log_prior.data_ptr() if log_prior is not None else None,
                              dlogits=None, row_loss=None, row_err=None)
                call("pkc_nll_fused", C.byref(a), s)
            else:
                a = L.DenseFwdArgs(
                    M=M, N=N, nslab=sf, zslab=zp, slab_stride=zs, bias=bias,
                    norm=(L.NORM_BN_TRAIN if train else L.NORM_BN_EVAL) if sp["bn"] else L.NORM_NONE,
                    gamma=sp["gamma"].data_ptr(), beta=sp["beta"].data_ptr(),
                    running_mean=sp["rm"].data_ptr(), running_var=sp["rv"].data_ptr(), momentum=0.05,
                    eps=1e-5, save_mean=b["sm"].data_ptr(), save_invstd=b["si"].data_ptr(),
                    act=L.ACT[sp["act"]], drop_p=0.0, seed=0, step_ctr=None, stream_id=0,
                    keep_in=None, keep_out=None, xhat=b["xhat"].data_ptr(), out=b["out"].data_ptr(),
                    count_n=0)
                call("pkc_dense_fwd", C.byref(a), ptr(b["work"]), s)
            cur, cld = b["out"].data_ptr(), N
        return self.bufs[-1]["out"][:M * self.bufs[-1]["N"]].view(M, -1)

    def forward(self, x, train=False):
        x = x.contiguous().float()
        return self.run(x.data_ptr(), x.shape[1], x.shape[0], train).clone()


class ForwardRunner:
    """run_nn forward mode (core.py:134-145, 234-249) for feed-forward models: one utterance per
    batch, BatchNorm with running statistics, no dropout, posteriors normalised by the log prior."""

    def __init__(self, nets, lines, fea_cols, forward_outs, max_rows=4096):
        fea_cols = resolve_concat(lines, fea_cols)
        self.lines, self.fea_cols, self.outs = lines, fea_cols, forward_outs
        self.nets = nets
        self.max_rows = max_rows
        self.runners = {}
        dims = {k: c1 - c0 for k, (c0, c1) in fea_cols.items()}
        for out, op, a, b in lines:
            if op == "compute":
                self.runners[a] = ModuleRunner(nets[a], max_rows, dims[b])
                dims[out] = nets[a].out_dim
        self.priors_dev = {}

    def forward(self, feats, beg, end, priors):
        M = end - beg
        if M > self.max_rows:
            raise ValueError("utterance of %d frames exceeds the forward buffer" % M)
        produced, res, cur = {}, {}, {}
        for out, op, a, b in self.lines:
            if op != "compute":
                continue
            if b in cur:                       # the version an earlier consumer quantised in place
                xp, ld = cur[b]
            elif b in self.fea_cols:
                c0, _ = self.fea_cols[b]
                xp, ld = feats.data_ptr() + 4 * (beg * feats.stride(0) + c0), feats.stride(0)
            else:
                xp, ld = produced[b].data_ptr(), produced[b].shape[1]
            lp = None
            if out in self.outs and out in priors:
                if out not in self.priors_dev:
                    self.priors_dev[out] = torch.from_numpy(priors[out]).to(feats.device)
                lp = self.priors_dev[out]
            y = self.runners[a].run(xp, ld, M, train=False, log_prior=lp)
            if self.runners[a].input_version is not None:
                cur[b] = (self.runners[a].input_version, ld)
            produced[out] = y
            if out in self.outs:
                res[out] = y.cpu().numpy()
            if all(o in res for o in self.outs):
                break
        return res
