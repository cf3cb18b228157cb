"""Trainable ``forward(x)`` of the architecture plug-ins (primary boundary).

The reference loads an architecture with ``cls(options, inp_dim)`` (utils.py:1768-1779), calls
``net(x)`` from utils.forward_model (utils.py:1884-2050) — x = (B, F) for a feed-forward arch, (T, B,
F) for a sequence arch — and trains it with ``loss.backward()`` + ``torch.optim`` (core.py:216-232).
pkc.neural_networks classes keep that contract: their ``forward`` is a torch.autograd.Function whose
forward and backward are the Engine's HIP layer kernels (pkc_gemm, pkc_dense_fwd/_bwd,
pkc_rnn_fwd/_bwd, pkc_logsoftmax_bwd ...) run in the Engine's external mode:

  * forward: the masks multiplied into W in place, prune, QuantizeLinear clamp + fake-quantised
    copy (as the reference does before every forward: neural_networks.py:256-278, 858-896), then
    the layer kernels over the caller's input;
  * backward: autograd's output gradient into the layer-backward kernels; every parameter's
    gradient comes back to autograd (accumulated into ``.grad`` like the reference's), and dL/dx
    when the input requires it (an MLP head over another arch's output).

No loss head and no optimizer run inside: the caller's NLLLoss and torch.optim do those, exactly
as with the reference classes.  Training-mode forward records state for ONE backward; calling the
same architecture again before that backward raises (the reference's forward_model calls each
architecture once per batch).  Eval mode (``net.eval()``) or ``torch.no_grad()``: forward only,
BatchNorm with running statistics, recurrent dropout as x(1-p).

In-place input fake-quantisation of the architecture's own input (``*_quant_inp`` with the first
layer reading x, QuantizeLinear.forward's ``input.data = Quantize_inp(input.data, ...)``,
quantized_modules.py:216-217, called by every gate projection of LSTM layer 0,
neural_networks.py:686-692, 948-951): the chain q1..qQ runs on the GPU (pkc_fakequant_input), each
gate's projection reads its own version, and the caller's tensor is rebound to the final version
(``x.data = qQ``) before ``forward`` returns, so later readers of the same tensor object see it,
as with the reference.  Autograd does not see the rebinding (the reference's is through
``.data`` too): dL/dx is the plain dX of layer 0.

Not supported here (raise NotImplementedError, run through pkc.core.run_nn instead): SyncBN.
"""
import torch

from . import _lib as L
from ._lib import call, ptr
from .engine import Engine

ARCH = "arch"


class ArchRunner:
    """External-mode Engine(s) of one architecture, rebuilt when a batch outgrows them."""

    def __init__(self, net):
        self.net = net
        self.seq = bool(getattr(net, "seq_model", False))
        self.eng = None
        self.gen = 0               # forward calls so far (a backward must follow its own)
        self.pending = None        # gen of the training forward whose state the buffers hold

    def _engine(self, rows, T, B, K):
        e = self.eng
        fits = (e is not None and e.F == K and
                (e.B == B and e.max_len >= T if self.seq else e.Mmax >= rows))
        if fits:
            return e
        dev = next(self.net.parameters()).device
        if self.seq:
            cap_T = max(T, 2 * e.max_len if (e is not None and e.B == B) else T)
            kw = dict(batch=B, max_len=cap_T)
        else:
            kw = dict(batch=max(rows, 2 * e.Mmax if e is not None else rows))
        lines = [["out", "compute", ARCH, "x"]]
        e = Engine({ARCH: self.net}, {ARCH: {}}, lines, {"x": (0, K)}, [], prec=L.PREC_FP32,
                   device=dev, seed=getattr(self.net, "pkc_seed", 0), external=True, **kw)
        if self.eng is not None:
            e.ctr.copy_(self.eng.ctr)      # keep the dropout streams advancing
        # nn.BatchNorm1d counts its training forwards (the kernels update the running statistics)
        self.nbt = []
        for n in e.nodes:
            if n.rec:
                self.nbt += [bn.num_batches_tracked for sp in n.layers if sp["bn"] for bn in sp["bnm"]]
            elif n.bn and n.spec.get("nbt") is not None:
                self.nbt.append(n.spec["nbt"])
        self.eng = e
        self.pending = None
        return e

    def forward(self, x, train):
        """x: (rows, K) or (T, B, K) fp32 on the device.  Returns (output, engine)."""
        if self.seq:
            if x.dim() != 3:
                raise ValueError("sequence architecture expects (T, B, F), got %s" % (tuple(x.shape),))
            T, B, K = x.shape
            rows = T * B
        else:
            if x.dim() != 2:
                raise ValueError("feed-forward architecture expects (B, F), got %s" % (tuple(x.shape),))
            rows, K = x.shape
            T, B = 1, rows
        e = self._engine(rows, T, B, K)
        xf = x.detach().contiguous()
        if xf.dtype != torch.float32:
            raise TypeError("pkc plug-in forward: fp32 input expected")
        if self.seq:
            e.T, e.M = T, rows
        else:
            e.M = rows
        e.x = xf.view(-1)              # the caller's input (held until the backward)
        s = Engine._stream()
        e.apply_weight_masks(s)
        e._forward_kernels(s, train)
        if train:
            e.ctr.add_(1)              # next step's dropout draws
            for t in self.nbt:
                t.add_(1)
        last = e.nodes[-1]
        N = last.N
        y = last.out[:rows * N].view(rows, N).clone()
        ent = e.qsrc.get(("fea", 0, K))
        if ent is not None and ent["Q"]:
            # quantized_modules.py:216-217: the caller's tensor now holds the last in-place version
            n = rows * K
            x.data = ent["buf"][(ent["Q"] - 1) * n:ent["Q"] * n].view(x.shape).clone()
        self.gen += 1
        self.pending = self.gen if train else None
        return (y.view(T, B, N) if self.seq else y), e

    def backward(self, gen, gy, want_dx):
        e = self.eng
        if self.pending != gen:
            raise RuntimeError("pkc plug-in: backward of a forward whose state was overwritten "
                               "(the architecture ran again, or was rebuilt, before this backward)")
        self.pending = None
        M = e.M
        last = e.nodes[-1]
        N = last.N
        gy = gy.contiguous().view(M, N)
        if gy.dtype != torch.float32:
            gy = gy.float()
        s = Engine._stream()
        e.gflat.zero_()
        e.want_dx = bool(want_dx)
        if last.head:                  # LogSoftmax output: its backward under this gradient
            call("pkc_logsoftmax_bwd", M, N, ptr(last.out), ptr(gy),
                 ptr(last.dz_ln if last.ln else last.dz), s)
        else:
            last.gsrc = (gy, 1, M * N)
        e._backward_kernels(s)
        e.want_dx = False
        grads = [g.clone() for _, g in e.param_grads]
        dx = None
        if want_dx:
            first = e.nodes[0]
            src = first.dz if (not first.rec and first.W is None) else e.ext_dx
            dx = src[:M * e.F].view(M, e.F).clone()
        return dx, grads


class _ArchFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, runner, x, *params):
        y, _ = runner.forward(x, True)
        ctx.runner, ctx.gen = runner, runner.gen
        ctx.xshape = x.shape
        ctx.save_for_backward(x)       # in-place changes of x before the backward are caught
        return y

    @staticmethod
    def backward(ctx, gy):
        ctx.saved_tensors
        dx, grads = ctx.runner.backward(ctx.gen, gy, ctx.needs_input_grad[1])
        if dx is not None:
            dx = dx.view(ctx.xshape)
        return (None, dx) + tuple(grads)


def arch_forward(net, x):
    """net(x) for a pkc.neural_networks architecture (see module docstring)."""
    r = getattr(net, "_pkc_runner", None)
    if r is None:
        r = net._pkc_runner = ArchRunner(net)
    if not x.is_cuda:
        raise RuntimeError("pkc plug-in forward: the input must be on the GPU (libpkc kernels)")
    train = net.training
    if not (train and torch.is_grad_enabled()):
        with torch.no_grad():
            y, _ = r.forward(x, train)
        return y
    # the engine (and so the parameter list) for this shape, before autograd sees the inputs
    if r.seq:
        T, B, K = x.shape
        r._engine(T * B, T, B, K)
    else:
        r._engine(x.shape[0], 1, x.shape[0], x.shape[1])
    params = [p for p, _ in r.eng.param_grads]
    return _ArchFunction.apply(r, x, *params)


def state_version(net):
    """Forward calls of net's plug-in runner so far (tests)."""
    r = getattr(net, "_pkc_runner", None)
    return 0 if r is None else r.gen


__all__ = ["arch_forward", "ArchRunner", "state_version"]
