"""pkc.engine — executes the cfg [model] graph of feed-forward (non-sequential) architectures on
the HIP kernels of libpkc.so.

What it replaces: core.run_nn's per-batch body (core.py:203-232) — utils.forward_model's
interpreter (utils.py:1884-2050) over MLP archs (neural_networks.py:245-319), the LogSoftmax +
NLLLoss + cost_err heads, autograd backward and the per-architecture optimizer steps.

Design (MI355X-first):
  * every tensor of a step lives in preallocated HBM buffers; a step is a fixed sequence of
    ~30 kernel launches on one stream (no host sync: loss/err accumulate on the device), which
    is captured once into a hipGraph (torch.cuda.CUDAGraph) and replayed per batch;
  * the batch is gathered from the HBM-resident chunk by a device-side batch counter, so graph
    replays walk the chunk without host involvement;
  * matmuls: pkc_gemm (MFMA, split-K slabs); BN/act/dropout fused in pkc_dense_fwd/_bwd;
    LogSoftmax+NLL+err+dlogits fused in pkc_nll_fused; all optimizers in one pkc_optim_step
    that also re-applies HCGS masks (the reference's in-place W.mul_(mask)).
"""
import ctypes as C
import re
import zlib

import numpy as np
import torch

from . import _lib as L
from ._lib import call, ptr

_PAT = re.compile(r"(.*)=(.*)\((.*),(.*)\)")


def parse_model(text):
    """utils.py:1888-1903 line grammar: out=op(in1,in2)."""
    return [list(_PAT.findall(line)[0]) for line in text.split("\n") if line.strip()]


def _f32(n, dev):
    return torch.zeros(int(n), dtype=torch.float32, device=dev)


class Layer:
    """One dense layer of an MLP architecture inside the graph."""

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
        self.src = None          # ("fea", c0, c1) or ("layer", Layer)
        self.consumers = []      # layers reading this output
        self.label_col = None    # head: label column index in the batch label buffer
        self.nbt0 = int(spec["nbt"].item()) if spec.get("nbt") is not None else 0
        self.loss_weight = 0.0
        self.name = "%s.%d" % (arch, idx)
        if self.head and self.bn:
            raise NotImplementedError("%s: BatchNorm before LogSoftmax is not on the pkc path" % self.name)
        if spec["ln"]:
            raise NotImplementedError("%s: LayerNorm is not on the pkc path yet" % self.name)
        if spec["quant"] or spec["inp_quant"]:
            raise NotImplementedError("%s: QuantizeLinear MLP layers are not on the pkc path yet"
                                      % self.name)
        if self.act not in L.ACT and not self.head:
            raise NotImplementedError("%s: activation %s" % (self.name, self.act))


class Engine:
    """Training / validation / forward executor of a non-sequential [model] graph.

    nets      : {arch_name: pkc.neural_networks.MLP} (parameters already on the device)
    arch_opts : {arch_name: configparser section} (optimizer + arch_freeze keys)
    lines     : parsed [model] lines
    fea_cols  : {fea_name: (c0, c1)} column range of each feature stream in the chunk matrix
    lab_names : ordered label names (label buffer column order)
    """

    def __init__(self, nets, arch_opts, lines, fea_cols, lab_names, batch, prec=L.PREC_FP32,
                 device="cuda", seed=0, train=True, drop_keep_in=None, grad_scale=1.0):
        self.dev = torch.device(device)
        self.nets, self.arch_opts, self.lines = nets, arch_opts, lines
        self.M = int(batch)
        self.prec = prec
        self.train = train
        self.seed = int(seed)
        self.grad_scale = float(grad_scale)   # 1/world_size under data parallelism
        self.prof = None                       # profile mode: list of per-launch events
        self.F = max(c1 for _, c1 in fea_cols.values())
        self.fea_cols = fea_cols
        self.lab_names = list(lab_names)
        self.nlab = len(self.lab_names)
        self._build_graph()
        self._alloc()
        self._build_optim()
        self.graph = None
        self.graph_opt = None
        self.steps_done = 0
        self.drop_keep_in = drop_keep_in or {}

    # ------------------------------------------------------------------ graph construction
    def _build_graph(self):
        self.layers, produced = [], {}
        for out, op, a, b in self.lines:
            if op != "compute":
                continue
            net = self.nets[a]
            net.check_supported()
            if b in self.fea_cols:
                src = ("fea",) + tuple(self.fea_cols[b])
                K = src[2] - src[1]
            elif b in produced:
                src = ("layer", produced[b])
                K = produced[b].N
            else:
                raise ValueError("input %s of %s is neither a feature nor a produced output" % (b, a))
            prev = src
            for i, spec in enumerate(net.layer_specs()):
                lay = Layer(a, i, spec, K)
                lay.src = prev
                if prev[0] == "layer":
                    prev[1].consumers.append(lay)
                self.layers.append(lay)
                prev = ("layer", lay)
                K = lay.N
                if lay.head and i != len(net.dnn_lay) - 1:
                    raise NotImplementedError("softmax only as the last layer of an MLP")
            produced[out] = prev[1]
        # loss expression (core.py uses loss_final / err_final)
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
            elif op == "compute":
                continue
            else:
                raise NotImplementedError("[model] operation %s is not on the pkc path" % op)
        self.heads = [l for l in self.layers if l.head]
        if self.train and "loss_final" not in scal:
            raise ValueError("[model] has no loss_final")
        for lay, w in scal.get("loss_final", {}).items():
            lay.loss_weight = w
        if self.err_layer is None and self.heads:
            self.err_layer = self.heads[0]
        for lay in self.layers:
            if lay.head and lay.label_col is None:
                lay.label_col = -1

    # ------------------------------------------------------------------ buffers
    def _alloc(self):
        M, dev = self.M, self.dev
        self.ctr = torch.zeros(2, dtype=torch.int64, device=dev)      # batch counter + done word
        self.x = _f32(M * self.F, dev)
        self.labs = torch.zeros(M * max(1, self.nlab), dtype=torch.int32, device=dev)
        for lay in self.layers:
            N, K = lay.N, lay.K
            lay.sf = L.lib().pkc_gemm_pick_splits(M, N, K)
            lay.zslab = _f32(lay.sf * M * N, dev)
            lay.out = _f32(M * N, dev)
            lay.xhat = None if lay.head else _f32(M * N, dev)
            lay.keep = torch.zeros(M * N, dtype=torch.uint8, device=dev) if lay.drop > 0 else None
            lay.save_mean = _f32(N, dev)
            lay.save_invstd = _f32(N, dev)
            lay.dz = _f32(M * N, dev)
            lay.work = _f32(L.lib().pkc_dense_work_size(M, N), dev)
            if lay.head:
                lay.row_loss = _f32(M, dev)
                lay.row_err = _f32(M, dev)
        for lay in self.layers:
            off = 0
            lay.cons_off = []
            for c in lay.consumers:
                s = L.lib().pkc_gemm_pick_splits(M, lay.N, c.N)
                c.sx = s
                lay.cons_off.append(off)
                off += s
            lay.sb = off
            lay.gslab = _f32(max(1, off) * M * lay.N, dev) if off else None
        self.needs_grad = {}
        for lay in reversed(self.layers):
            self.needs_grad[lay] = (lay.head and lay.loss_weight != 0.0) or any(
                self.needs_grad[c] for c in lay.consumers)
        # all gradients in ONE flat buffer (a single RCCL all-reduce under data parallelism)
        total = 0
        for lay in self.layers:
            total += lay.W.numel() + lay.b.numel() + (2 * lay.gamma.numel() if lay.bn else 0)
        self.gflat = _f32(total, dev)
        off = 0

        def take(like):
            nonlocal off
            t = self.gflat[off:off + like.numel()].view_as(like)
            off += like.numel()
            return t
        for lay in self.layers:
            lay.dW, lay.db = take(lay.W), take(lay.b)
            lay.dgamma = take(lay.gamma) if lay.bn else None
            lay.dbeta = take(lay.beta) if lay.bn else None
        # loss finalize descriptors
        self.loss_heads = [l for l in self.heads if l.label_col >= 0]
        if self.loss_heads:
            if self.err_layer not in self.loss_heads:
                raise NotImplementedError("err head without labels")
            self.loss_out = _f32(2 + len(self.loss_heads), dev)
            self.loss_acc = _f32(2, dev)
            ptrs = np.array([l.row_loss.data_ptr() for l in self.loss_heads], dtype=np.uint64)
            self.loss_ptrs = torch.from_numpy(ptrs.view(np.int64)).to(dev)
            self.loss_w = torch.tensor([l.loss_weight for l in self.loss_heads], dtype=torch.float32,
                                       device=dev)

    def _build_optim(self):
        """One pkc_opt_tensor per parameter that receives a gradient (utils.py:1833-1881)."""
        self.opt_entries = []   # (arch, param tensor, grad, state dict)
        for lay in self.layers:
            if not self.needs_grad[lay]:
                continue
            o = self.arch_opts[lay.arch]
            from .neural_networks import strtobool
            if strtobool(o.get("arch_freeze", "False")):
                continue
            plist = [(lay.W, lay.dW, lay.mask), (lay.b, lay.db, None)]
            if lay.bn:
                plist += [(lay.gamma, lay.dgamma, None), (lay.beta, lay.dbeta, None)]
            for p, g, m in plist:
                self.opt_entries.append(dict(arch=lay.arch, p=p, g=g, mask=m, o=o,
                                             s1=torch.zeros_like(p), s2=None, s3=None, step=0))
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
        if n:
            sizes = (C.c_int64 * n)(*[e["p"].numel() for e in self.opt_entries])
            nch = L.lib().pkc_optim_chunks(sizes, n, None, 0)
            cmap = (C.c_int32 * (2 * nch))()
            L.lib().pkc_optim_chunks(sizes, n, cmap, nch)
            self.opt_nchunks = nch
            self.opt_map = torch.from_numpy(np.frombuffer(cmap, dtype=np.int32).copy()).to(self.dev)
            self.opt_desc = torch.zeros(n * C.sizeof(L.OptTensor), dtype=torch.uint8, device=self.dev)
            self._upload_opt_desc(step_inc=1)
        # the reference multiplies the masks in before the first forward; do it once here
        for lay in self.layers:
            if lay.mask is not None:
                call("pkc_apply_mask", ptr(lay.W), ptr(lay.mask), lay.W.numel(), C.c_float(0.0),
                     self._stream())

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
            t.clampv = 0.0
            t.step = e["step"] + step_inc
        host = torch.frombuffer(bytearray(C.string_at(arr, C.sizeof(arr))), dtype=torch.uint8)
        self.opt_desc.copy_(host)

    def set_lr(self, arch, lr):
        for e in self.opt_entries:
            if e["arch"] == arch:
                e["o"] = dict(e["o"], arch_lr=str(lr))
        if self.opt_entries:
            self._upload_opt_desc(step_inc=1)

    # ------------------------------------------------------------------ chunk binding
    def bind_chunk(self, feats, labels, n_rows):
        """feats: (N, F) fp32 device tensor (row stride >= F); labels: (N, nlab) int32 device."""
        assert feats.dtype == torch.float32 and labels.dtype == torch.int32
        assert feats.shape[1] >= self.F and labels.shape[1] == self.nlab
        self.chunk_feats, self.chunk_labels = feats, labels
        self.n_batches = int(n_rows) // self.M
        self.ctr.zero_()
        if self.loss_heads:
            self.loss_acc.zero_()

    # ------------------------------------------------------------------ kernels of one step
    @staticmethod
    def _stream():
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def _k(self, label, flops, nbytes, fn, *args):
        """Launch one libpkc entry point; in profile mode bracket it with events."""
        if self.prof is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            call(fn, *args)
            e1.record()
            self.prof.append((label, fn, float(flops), float(nbytes), e0, e1))
        else:
            call(fn, *args)

    def _src(self, lay):
        if lay.src[0] == "fea":
            return self.x.data_ptr() + 4 * lay.src[1], self.F
        return lay.src[1].out.data_ptr(), lay.src[1].N

    def _forward_kernels(self, s, train):
        M = self.M
        self._k("batch_gather", 0, 8.0 * M * self.F, "pkc_batch_gather", ptr(self.chunk_feats),
                self.chunk_feats.stride(0), self.F, ptr(self.chunk_labels), self.nlab, M,
                self.n_batches, ptr(self.ctr), ptr(self.x), ptr(self.labs), 1, s)
        for lay in self.layers:
            a_ptr, lda = self._src(lay)
            self._k("gemm_fwd %dx%dx%d" % (M, lay.N, lay.K), 2.0 * M * lay.N * lay.K,
                    4.0 * (M * lay.K + lay.N * lay.K + lay.sf * M * lay.N), "pkc_gemm", self.prec,
                    1, 1, M, lay.N, lay.K, C.c_void_p(a_ptr), lda, ptr(lay.W), lay.K, ptr(lay.zslab),
                    lay.N, lay.sf, M * lay.N, s)
            if lay.head:
                has_lab = lay.label_col >= 0
                a = L.NllArgs(M=M, N=lay.N, nslab=lay.sf, zslab=lay.zslab.data_ptr(),
                              slab_stride=M * lay.N, bias=lay.b.data_ptr(),
                              labels=(self.labs.data_ptr() + 4 * lay.label_col) if has_lab else None,
                              label_stride=self.nlab, weight=lay.loss_weight * self.grad_scale,
                              logp=lay.out.data_ptr(),
                              log_prior=None,
                              dlogits=lay.dz.data_ptr() if (train and has_lab) else None,
                              row_loss=lay.row_loss.data_ptr(), row_err=lay.row_err.data_ptr())
                self._k("nll_fused N=%d" % lay.N, 0, 4.0 * M * lay.N * (lay.sf + 2), "pkc_nll_fused",
                        C.byref(a), s)
            else:
                keep_in = self.drop_keep_in.get(lay.name)
                a = L.DenseFwdArgs(
                    M=M, N=lay.N, nslab=lay.sf, zslab=lay.zslab.data_ptr(), slab_stride=M * lay.N,
                    bias=lay.b.data_ptr(),
                    norm=(L.NORM_BN_TRAIN if train else L.NORM_BN_EVAL) if lay.bn else L.NORM_NONE,
                    gamma=lay.gamma.data_ptr(), beta=lay.beta.data_ptr(),
                    running_mean=lay.rm.data_ptr(), running_var=lay.rv.data_ptr(),
                    momentum=0.05, eps=1e-5, save_mean=lay.save_mean.data_ptr(),
                    save_invstd=lay.save_invstd.data_ptr(), act=L.ACT[lay.act],
                    drop_p=lay.drop if train else 0.0, seed=self.seed,
                    step_ctr=self.ctr.data_ptr(), stream_id=zlib.crc32(lay.name.encode()),
                    keep_in=keep_in.data_ptr() if keep_in is not None else None,
                    keep_out=lay.keep.data_ptr() if (lay.keep is not None and train) else None,
                    xhat=lay.xhat.data_ptr(), out=lay.out.data_ptr())
                self._k("dense_fwd N=%d" % lay.N, 0, 4.0 * M * lay.N * (lay.sf + 2), "pkc_dense_fwd",
                        C.byref(a), ptr(lay.work), s)
        if self.loss_heads:
            err_out = self.err_layer.row_err
            self._k("loss_finalize", 0, 4.0 * M * (len(self.loss_heads) + 1), "pkc_loss_finalize",
                    len(self.loss_heads), ptr(self.loss_ptrs), ptr(self.loss_w), M, ptr(err_out),
                    ptr(self.loss_out), ptr(self.loss_acc), s)

    def _backward_kernels(self, s):
        M = self.M
        for lay in reversed(self.layers):
            if not self.needs_grad[lay]:
                continue
            if lay.head:
                self._k("colsum N=%d" % lay.N, 0, 4.0 * M * lay.N, "pkc_colsum", M, lay.N, 1,
                        ptr(lay.dz), 0, ptr(lay.db), 0, s)
            else:
                a = L.DenseBwdArgs(M=M, N=lay.N, nslab=lay.sb, gslab=lay.gslab.data_ptr(),
                                   slab_stride=M * lay.N,
                                   norm=L.NORM_BN_TRAIN if lay.bn else L.NORM_NONE,
                                   act=L.ACT[lay.act], gamma=lay.gamma.data_ptr(),
                                   beta=lay.beta.data_ptr(), save_invstd=lay.save_invstd.data_ptr(),
                                   xhat=lay.xhat.data_ptr(),
                                   keep=lay.keep.data_ptr() if lay.keep is not None else None,
                                   drop_p=lay.drop, dz=lay.dz.data_ptr(),
                                   dgamma=lay.dgamma.data_ptr() if lay.bn else None,
                                   dbeta=lay.dbeta.data_ptr() if lay.bn else None,
                                   dbias=lay.db.data_ptr())
                self._k("dense_bwd N=%d" % lay.N, 0, 4.0 * M * lay.N * (lay.sb + 3), "pkc_dense_bwd",
                        C.byref(a), ptr(lay.work), s)
            a_ptr, lda = self._src(lay)
            # dW = dz^T X
            self._k("gemm_dW %dx%dx%d" % (lay.N, lay.K, M), 2.0 * M * lay.N * lay.K,
                    4.0 * (M * lay.N + M * lay.K + lay.N * lay.K), "pkc_gemm", self.prec, 0, 0,
                    lay.N, lay.K, M, ptr(lay.dz), lay.N, C.c_void_p(a_ptr), lda, ptr(lay.dW), lay.K,
                    1, 0, s)
            if lay.src[0] == "layer" and self.needs_grad[lay.src[1]]:
                P = lay.src[1]
                off = P.cons_off[P.consumers.index(lay)]
                # dX slabs = dz W into the producer's gradient slabs
                self._k("gemm_dX %dx%dx%d" % (M, lay.K, lay.N), 2.0 * M * lay.N * lay.K,
                        4.0 * (M * lay.N + lay.N * lay.K + lay.sx * M * lay.K), "pkc_gemm",
                        self.prec, 1, 0, M, lay.K, lay.N, ptr(lay.dz), lay.N, ptr(lay.W), lay.K,
                        C.c_void_p(P.gslab.data_ptr() + 4 * off * M * P.N), lay.K, lay.sx,
                        M * lay.K, s)

    def _optim_kernels(self, s):
        if self.opt_entries:
            nparam = sum(e["p"].numel() for e in self.opt_entries)
            self._k("optim_step", 0, 4.0 * nparam * 5, "pkc_optim_step", ptr(self.opt_desc),
                    len(self.opt_entries), ptr(self.opt_map), self.opt_nchunks, s)

    def _train_step_kernels(self, allreduce=None):
        s = self._stream()
        self._forward_kernels(s, True)
        self._backward_kernels(s)
        if allreduce is not None:
            allreduce(self.gflat)
        self._optim_kernels(s)

    # ------------------------------------------------------------------ public API
    def train_step(self, allreduce=None):
        """One batch: forward, backward, [allreduce(flat grads)], optimizer (core.py:216-232)."""
        if self.graph is not None:
            self.graph.replay()
            if self.graph_opt is not None:
                if allreduce is not None:
                    allreduce(self.gflat)
                self.graph_opt.replay()
        else:
            self._train_step_kernels(allreduce)
        self._after_step()

    def profile_step(self):
        """Run one eager training step with events around every launch; returns
        [(label, fn, flops, bytes, ms)] (device time per launch)."""
        self.prof = []
        self._train_step_kernels()
        torch.cuda.synchronize()
        out = [(l, f, fl, nb, e0.elapsed_time(e1)) for (l, f, fl, nb, e0, e1) in self.prof]
        self.prof = None
        self._after_step()
        return out

    def _after_step(self):
        self.steps_done += 1
        for e in self.opt_entries:
            e["step"] += 1
        if self.opt_entries and not self.static_opt and self.graph is None:
            self._upload_opt_desc(step_inc=1)

    def capture(self, split_optimizer=False):
        """Capture the training step into hipGraph(s) (needs step-independent optimizer
        descriptors: RMSprop / momentum-free SGD).  split_optimizer=True captures forward+backward
        and the optimizer separately so a gradient all-reduce can run in between."""
        if not self.static_opt:
            return False
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            st = self._stream()
            self._forward_kernels(st, True)
            self._backward_kernels(st)
            if not split_optimizer:
                self._optim_kernels(st)
        self.graph_opt = None
        if split_optimizer:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, stream=s):
                self._optim_kernels(self._stream())
            self.graph_opt = g2
        torch.cuda.current_stream().wait_stream(s)
        self.graph = g
        return True

    def eval_step(self):
        """Validation batch: forward with running BN statistics, loss/err accumulated."""
        self._forward_kernels(self._stream(), False)

    def loss_values(self):
        """(loss_final, err) of the last step (forces a sync)."""
        v = self.loss_out.cpu()
        return float(v[0]), float(v[1])

    def chunk_totals(self):
        """(loss_sum, err_sum) over the batches since bind_chunk (core.py:251-252)."""
        v = self.loss_acc.cpu()
        return float(v[0]), float(v[1])

    def sync_state(self):
        """Reflect the step count into BN num_batches_tracked (nn.BatchNorm1d increments it on
        every training forward; the kernels update running stats but not this counter)."""
        for lay in self.layers:
            if lay.bn:
                lay.spec["nbt"].fill_(lay.nbt0 + self.steps_done)

    def optimizer_state_dict(self, arch):
        """torch.optim-compatible state_dict of one architecture's optimizer (core.py:317-322)."""
        net = self.nets[arch]
        params = list(net.parameters())
        index = {id(p): i for i, p in enumerate(params)}
        o = self.arch_opts[arch]
        state = {}
        for e in self.opt_entries:
            if e["arch"] != arch or e["step"] == 0:
                continue
            st = {"step": torch.tensor(float(e["step"]))}
            kind = o["arch_opt"]
            if kind == "rmsprop":
                st["square_avg"] = e["s1"].detach().cpu().clone()
                if e["s3"] is not None:
                    st["momentum_buffer"] = e["s3"].detach().cpu().clone()
                if e["s2"] is not None:
                    st["grad_avg"] = e["s2"].detach().cpu().clone()
            elif kind == "sgd":
                st = {"momentum_buffer": e["s1"].detach().cpu().clone()
                      if float(o["opt_momentum"]) != 0 else None}
            else:
                st["exp_avg"] = e["s1"].detach().cpu().clone()
                st["exp_avg_sq"] = e["s2"].detach().cpu().clone()
            state[index[id(e["p"])]] = st
        group = {"params": list(range(len(params))), "lr": float(o["arch_lr"])}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, arch, sd):
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
            if "exp_avg" in st:
                e["s1"].copy_(st["exp_avg"])
                e["s2"].copy_(st["exp_avg_sq"])
            if st.get("momentum_buffer") is not None:
                (e["s3"] if e["s3"] is not None else e["s1"]).copy_(st["momentum_buffer"])
            if "step" in st:
                e["step"] = int(float(st["step"]))
        self._upload_opt_desc(step_inc=1)


def _b(v):
    return str(v).strip().lower() in ("1", "true", "yes", "y", "on", "t")


class ModuleRunner:
    """Forward of one MLP module on the pkc kernels for any row count <= max_rows (MLP.forward for
    stand-alone calls, and the per-utterance forward of run_nn's forward mode)."""

    def __init__(self, net, max_rows, inp_dim):
        net.check_supported()
        self.net, self.rows, self.dev = net, max_rows, next(net.parameters()).device
        self.specs = net.layer_specs()
        self.bufs = []
        K = inp_dim
        for sp in self.specs:
            N = sp["out"]
            sf = L.lib().pkc_gemm_pick_splits(max_rows, N, K)
            self.bufs.append(dict(sf=sf, z=_f32(sf * max_rows * N, self.dev), K=K, N=N,
                                  xhat=_f32(max_rows * N, self.dev), sm=_f32(N, self.dev),
                                  si=_f32(N, self.dev), out=_f32(max_rows * N, self.dev),
                                  work=_f32(L.lib().pkc_dense_work_size(max_rows, N), self.dev)))
            K = N
        for sp in self.specs:
            if sp["mask"] is not None:
                call("pkc_apply_mask", ptr(sp["W"]), ptr(sp["mask"]), sp["W"].numel(),
                     C.c_float(0.0), Engine._stream())

    def run(self, x_ptr, ld, M, train=False, log_prior=None):
        """x_ptr: device address of an (M, ld) fp32 matrix; returns the (M, N) output view."""
        assert M <= self.rows
        s = Engine._stream()
        cur, cld = x_ptr, ld
        for sp, b in zip(self.specs, self.bufs):
            N, K = b["N"], b["K"]
            sf = L.lib().pkc_gemm_pick_splits(M, N, K)
            call("pkc_gemm", L.PREC_FP32, 1, 1, M, N, K, C.c_void_p(cur), cld, ptr(sp["W"]), K,
                 ptr(b["z"]), N, sf, M * N, s)
            if sp["act"] == "softmax":
                a = L.NllArgs(M=M, N=N, nslab=sf, zslab=b["z"].data_ptr(), slab_stride=M * N,
                              bias=sp["b"].data_ptr(), labels=None, label_stride=0, weight=0.0,
                              logp=b["out"].data_ptr(),
                              log_prior=log_prior.data_ptr() if log_prior is not None else None,
                              dlogits=None, row_loss=None, row_err=None)
                call("pkc_nll_fused", C.byref(a), s)
            else:
                a = L.DenseFwdArgs(
                    M=M, N=N, nslab=sf, zslab=b["z"].data_ptr(), slab_stride=M * N,
                    bias=sp["b"].data_ptr(),
                    norm=(L.NORM_BN_TRAIN if train else L.NORM_BN_EVAL) if sp["bn"] else L.NORM_NONE,
                    gamma=sp["gamma"].data_ptr(), beta=sp["beta"].data_ptr(),
                    running_mean=sp["rm"].data_ptr(), running_var=sp["rv"].data_ptr(), momentum=0.05,
                    eps=1e-5, save_mean=b["sm"].data_ptr(), save_invstd=b["si"].data_ptr(),
                    act=L.ACT[sp["act"]], drop_p=0.0, seed=0, step_ctr=None, stream_id=0,
                    keep_in=None, keep_out=None, xhat=b["xhat"].data_ptr(), out=b["out"].data_ptr())
                call("pkc_dense_fwd", C.byref(a), ptr(b["work"]), s)
            cur, cld = b["out"].data_ptr(), N
        return self.bufs[-1]["out"][:M * self.bufs[-1]["N"]].view(M, -1)

    def forward(self, x, train=False):
        x = x.contiguous().float()
        return self.run(x.data_ptr(), x.shape[1], x.shape[0], train).clone()


class ForwardRunner:
    """run_nn forward mode (core.py:134-145, 234-249): one utterance per batch, BatchNorm with
    running statistics, no dropout, posteriors normalised by the log class prior."""

    def __init__(self, nets, lines, fea_cols, forward_outs, max_rows=4096):
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
        produced, res = {}, {}
        for out, op, a, b in self.lines:
            if op != "compute":
                continue
            if b in self.fea_cols:
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
            produced[out] = y
            if out in self.outs:
                res[out] = y.cpu().numpy()
            if all(o in res for o in self.outs):
                break
        return res
