"""Drop-in architecture plug-ins: ``arch_library = pkc.neural_networks``, ``arch_class = MLP``.

Loaded exactly like the reference's classes (utils.py:1766-1779:
``getattr(importlib.import_module(arch_library), arch_class)(options, inp_dim)``) and exposing the
same contract: ``.out_dim``, ``forward(x)``, ``parameters()/state_dict()/load_state_dict()``,
``train()/eval()``, and the attributes core.run_nn reads (``prune``, ``prune_parameters()``,
``guided_hcgs``, ``apply_guided_hcgs``, ``if_pattern``, ``skip_regularization``).

Parameter names, shapes and the construction-time RNG consumption follow neural_networks.py:81-243
so a state_dict / .pkl checkpoint moves between the reference and this package unchanged and the
same seed gives the same initial weights and HCGS masks.

The math is NOT executed here: training and forward passes run through pkc.engine (HIP kernels in
libpkc.so), driven by pkc.core.run_nn, or by ``forward()`` below — an autograd Function over the
same kernels (pkc.plugin), so the reference's own forward_model + loss.backward() + torch.optim
loop (utils.py:1884-2050, core.py:216-232) trains these classes too.
"""
import math

import numpy as np
import torch
import torch.nn as nn

from .cgs import guided_hcgs_mask, hcgs_mask
from .plugin import arch_forward


def strtobool(v):
    v = str(v).strip().lower()
    if v in ("y", "yes", "t", "true", "on", "1"):
        return 1
    if v in ("n", "no", "f", "false", "off", "0"):
        return 0
    raise ValueError("invalid truth value %r" % v)


def _lst(opts, key, f=str):
    return [f(x) for x in opts[key].split(",")]


class LayerNorm(nn.Module):
    """Parameter holder with the reference's names (neural_networks.py:40-51)."""

    def __init__(self, features, eps=1e-6):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(features))
        self.beta = nn.Parameter(torch.zeros(features))
        self.eps = eps


def _prune_params(params, perc):
    """quantized_modules.prune + W.mul_(mask) on each parameter, on the GPU (pkc_prune)."""
    import ctypes as C
    from . import _lib as L
    work = torch.zeros(L.lib().pkc_prune_work_size(), dtype=torch.uint8, device=params[0].device)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for p in params:
        L.call("pkc_prune", L.ptr(p.data), p.numel(), C.c_double(perc), None, L.ptr(work), s)
    torch.cuda.synchronize()


def _input_norm_specs(net, ln, bn):
    """ln0 (per row) then bn0 (over all rows; T*B rows, padding included, for a recurrent
    architecture: neural_networks.py:826-831) as engine NormLayer specs."""
    out = []
    if ln:
        out.append(dict(kind="ln", gamma=net.ln0.gamma, beta=net.ln0.beta))
    if bn:
        out.append(dict(kind="bn", gamma=net.bn0.weight, beta=net.bn0.bias,
                        rm=net.bn0.running_mean, rv=net.bn0.running_var,
                        nbt=net.bn0.num_batches_tracked))
    return out


class _PatternSet:
    """Pattern-set plumbing shared by MLP and LSTM (neural_networks.py:115-131, 513-529).
    A set comes from ``pattern_from_file`` / ``pattern_file`` (an (P*ph, pw) .npy such as
    pattern_file/b08b08_k04_n16_pattern.npy; a pkc option, shared by every weight), from
    ``pattern_kernels = ...``, or from the ``patterns`` dict run_nn carries between chunks
    (core.py:129-131, 304-306).  Without one, each weight's set is searched as the reference does
    (update_patterns -> sparsity.find_top_k_by_kmeans with pattern_num / pattern_nnz per layer,
    neural_networks.py:339-348, 1162-1172; ``pkc.cgs.kmeans_patterns``): sklearn KMeans with no
    random_state, so parity is unpinned unless ``pattern_seed`` is given."""

    def _pattern_opts(self, o):
        self.if_pattern = strtobool(o["if_pattern"]) if "if_pattern" in o else False
        self.pattern_shape = _lst(o, "pattern_shape", int) if "pattern_shape" in o else [8, 8]
        self.pattern_from_file = o.get("pattern_from_file", o.get("pattern_file", None))
        self.pattern_nnz = _lst(o, "pattern_nnz", int) if "pattern_nnz" in o else []
        self.pattern_num = _lst(o, "pattern_num", int) if "pattern_num" in o else []
        self.pattern_seed = int(o["pattern_seed"]) if "pattern_seed" in o else None

    def can_search_patterns(self):
        return bool(self.pattern_nnz) and bool(self.pattern_num)

    def pattern_search_args(self, layer):
        """(pattern_num, pattern_shape, pattern_nnz) of layer ``layer`` (neural_networks.py:344)."""
        return (self.pattern_num[min(layer, len(self.pattern_num) - 1)], list(self.pattern_shape),
                self.pattern_nnz[min(layer, len(self.pattern_nnz) - 1)])

    @property
    def pattern_kernels(self):
        """(P, ph, pw) float32 pattern set, or None."""
        k = getattr(self, "_pattern_kernels", None)
        if k is None and self.if_pattern:
            pat = self.pattern
            first = (pat[0] if isinstance(pat, list) and pat else
                     next((v[0] for v in pat.values() if v), None) if isinstance(pat, dict) else None)
            if first is not None:                   # (P, 1, ph, pw) kernel, as the reference keeps
                t = first.detach().cpu().numpy() if torch.is_tensor(first) else np.asarray(first)
                k = t.reshape(t.shape[0], t.shape[-2], t.shape[-1]).astype(np.float32)
            elif self.pattern_from_file:
                arr = np.load(self.pattern_from_file, allow_pickle=False).astype(np.float32)
                ph, pw = self.pattern_shape
                k = arr.reshape(-1, ph, pw)
            self._pattern_kernels = k
        return k

    @pattern_kernels.setter
    def pattern_kernels(self, v):
        self._pattern_kernels = None if v is None else np.asarray(v, dtype=np.float32)


class _Mask(nn.Module):
    """HCGS.HCGS / HCGS.guidedHCGS: a ``mask`` Parameter of shape (out, in) (HCGS.py:24-28, 55-59)."""

    def __init__(self, mask):
        super().__init__()
        self.mask = nn.Parameter(torch.from_numpy(mask))


def _mask_product(*ms):
    """Effective in-place mask of several masks multiplied into W one after the other."""
    ms = [m for m in ms if m is not None]
    if not ms:
        return None
    out = ms[0]
    for m in ms[1:]:
        out = out * m
    return out.detach() if len(ms) > 1 else out


def _set_mask(module, arr):
    module.mask.data.copy_(torch.from_numpy(arr).to(module.mask.device))


class _QLinear(nn.Module):
    """Parameter layout + init draws of QuantizeLinear (quantized_modules.py:184-205)."""

    def __init__(self, fin, fout, bits, bias, inp_bits=None):
        super().__init__()
        self.weight = nn.Parameter(torch.Tensor(fout, fin))
        self.bias = nn.Parameter(torch.Tensor(fout)) if bias else None
        s = 1.0 / math.sqrt(fin)
        self.weight.data.uniform_(-s, s)
        if self.bias is not None:
            self.bias.data.uniform_(-s, s)
        self.numBits = bits
        self.inp_quant = inp_bits


class MLP(_PatternSet, nn.Module):
    """neural_networks.py:81-361 (options per proto/MLP.proto + the CGS keys)."""

    seq_model = False

    def __init__(self, options, inp_dim):
        super().__init__()
        o = options
        self.input_dim = inp_dim
        self.dnn_lay = _lst(o, "dnn_lay", int)
        self.dnn_drop = _lst(o, "dnn_drop", float)
        self.dnn_use_batchnorm = _lst(o, "dnn_use_batchnorm", strtobool)
        self.dnn_use_laynorm = _lst(o, "dnn_use_laynorm", strtobool)
        self.dnn_use_laynorm_inp = strtobool(o["dnn_use_laynorm_inp"])
        self.dnn_use_batchnorm_inp = strtobool(o["dnn_use_batchnorm_inp"])
        self.dnn_act = _lst(o, "dnn_act")
        self.to_do = o.get("to_do", "train")
        self.mlp_hcgs = strtobool(o.get("mlp_hcgs", "False"))
        self.hcgs_block = _lst(o, "hcgs_block", int) if "hcgs_block" in o else []
        self.hcgs_sparse = _lst(o, "hcgs_sparse", float) if "hcgs_sparse" in o else []
        self.mlp_quant = strtobool(o.get("mlp_quant", "False"))
        self.param_quant = _lst(o, "param_quant", int) if "param_quant" in o else [8]
        self.mlp_quant_inp = strtobool(o.get("mlp_quant_inp", "False"))
        self.inp_quant = _lst(o, "inp_quant", int) if "inp_quant" in o else [16]
        self.prune = strtobool(o.get("mlp_prune", "False"))
        self.prune_perc = _lst(o, "mlp_prune_perc", float) if "mlp_prune_perc" in o else [0.0]
        self.skip_regularization = strtobool(o.get("skip_regularization", "False"))
        self.guided_hcgs = strtobool(o.get("guided_hcgs", "False"))
        self.apply_guided_hcgs = strtobool(o.get("apply_guided_hcgs", "False"))
        self._pattern_opts(o)
        self.arch_name = o.get("arch_name", "MLP")
        if self.if_pattern:                  # per-layer kernels / masks (neural_networks.py:159-161)
            self.pattern, self.pattern_mask = [], []

        if self.mlp_hcgs:                    # registered first, as neural_networks.py:151-156
            self.hcgs = nn.ModuleList()
        if self.guided_hcgs:
            self.ghcgs = nn.ModuleList()
        self.wx, self.bn, self.ln = nn.ModuleList(), nn.ModuleList(), nn.ModuleList()
        if self.dnn_use_laynorm_inp:
            self.ln0 = LayerNorm(inp_dim)
        if self.dnn_use_batchnorm_inp:
            self.bn0 = nn.BatchNorm1d(inp_dim, momentum=0.05)
        cur = inp_dim
        for i, n in enumerate(self.dnn_lay):
            self.ln.append(LayerNorm(n))
            self.bn.append(nn.BatchNorm1d(n, momentum=0.05))
            add_bias = not (self.dnn_use_laynorm[i] or self.dnn_use_batchnorm[i])
            if self.mlp_quant:
                lin = _QLinear(cur, n, self.param_quant[i], add_bias,
                               self.inp_quant[0] if self.mlp_quant_inp else None)
            else:
                lin = nn.Linear(cur, n, bias=add_bias)          # consumes the torch RNG as the ref
            self.wx.append(lin)
            if self.mlp_hcgs:
                self.hcgs.append(_Mask(hcgs_mask(n, cur, self.hcgs_block, self.hcgs_sparse)))
            s = np.sqrt(0.01 / (cur + n))                        # neural_networks.py:233-235
            lin.weight = nn.Parameter(torch.Tensor(n, cur).uniform_(-s, s))
            lin.bias = nn.Parameter(torch.zeros(n))
            if self.guided_hcgs:             # from the initial W (neural_networks.py:237-239)
                self.ghcgs.append(_Mask(guided_hcgs_mask(n, cur, self.hcgs_block, self.hcgs_sparse,
                                                         lin.weight.data)))
            cur = n
        self.out_dim = cur

    # --------------------------------------------------------------------- reference hooks
    def prune_parameters(self):
        """Chunk-end pruning (neural_networks.py:321-327, called at core.py:291-296): every
        layer's W pruned at prune_perc[0] (the reference uses the first entry for all layers)."""
        _prune_params([self.wx[i].weight for i in range(len(self.dnn_lay))], self.prune_perc[0])
        return 1

    def apply_ghcgs(self):
        """Chunk-end regeneration of the guided masks from the current W (neural_networks.py:
        329-337, called at core.py:298-300 while apply_guided_hcgs is off)."""
        cur = self.input_dim
        for i, n in enumerate(self.dnn_lay):
            _set_mask(self.ghcgs[i], guided_hcgs_mask(n, cur, self.hcgs_block, self.hcgs_sparse,
                                                      self.wx[i].weight.data))
            cur = n
        return 20.0

    def _wmask(self, i):
        """Masks multiplied into wx[i] before each forward: HCGS, then guided HCGS when applied
        (neural_networks.py:256-262)."""
        return _mask_product(self.hcgs[i].mask if self.mlp_hcgs else None,
                             self.ghcgs[i].mask if (self.guided_hcgs and self.apply_guided_hcgs)
                             else None)

    def layer_specs(self):
        """Per-layer description consumed by pkc.engine."""
        specs = []
        for i, n in enumerate(self.dnn_lay):
            specs.append(dict(out=n, act=self.dnn_act[i], bn=bool(self.dnn_use_batchnorm[i]),
                              ln=bool(self.dnn_use_laynorm[i]), drop=self.dnn_drop[i],
                              W=self.wx[i].weight, b=self.wx[i].bias, gamma=self.bn[i].weight,
                              beta=self.bn[i].bias, rm=self.bn[i].running_mean,
                              rv=self.bn[i].running_var, nbt=self.bn[i].num_batches_tracked,
                              mask=self._wmask(i),
                              quant=self.param_quant[i] if self.mlp_quant else 0,
                              inp_quant=self.inp_quant[0] if (self.mlp_quant and self.mlp_quant_inp) else 0,
                              ln_gamma=self.ln[i].gamma, ln_beta=self.ln[i].beta,
                              prune=self.prune_perc[i] if self.prune else None,
                              pattern=bool(self.if_pattern)))
        return specs

    def pattern_params(self):
        """[(store key, layer, W, HCGS mask)] in the reference's update_mask order."""
        return [((None, i), i, self.wx[i].weight, self._wmask(i)) for i in range(len(self.dnn_lay))]

    def input_norm_specs(self):
        """Input normalisations in the reference's order: ln0 then bn0 (neural_networks.py:246-251)."""
        return _input_norm_specs(self, self.dnn_use_laynorm_inp, self.dnn_use_batchnorm_inp)

    def check_supported(self):
        if self.if_pattern and self.pattern_kernels is None and not self.can_search_patterns():
            raise NotImplementedError("pattern MLP needs a pattern set (pattern_from_file option, "
                                      "pattern_kernels, patterns injected by run_nn) or "
                                      "pattern_num / pattern_nnz for the KMeans search")

    def forward(self, x):
        """(B, F) -> (B, out_dim) on the pkc kernels, trainable under autograd (pkc.plugin)."""
        return arch_forward(self, x)


class liGRU(nn.Module):
    """neural_networks.py:1429-1599 (options per proto/liGRU.proto).  Parameters: wh, wz (input
    Linear), uh, uz (recurrent Linear, no bias), bn_wh, bn_wz, ln; same names and init draws."""

    seq_model = True
    cell = "ligru"
    GATES = ("z", "h")

    def __init__(self, options, inp_dim):
        super().__init__()
        o = options
        self.input_dim = inp_dim
        self.ligru_lay = _lst(o, "ligru_lay", int)
        self.ligru_drop = _lst(o, "ligru_drop", float)
        self.ligru_use_batchnorm = _lst(o, "ligru_use_batchnorm", strtobool)
        self.ligru_use_laynorm = _lst(o, "ligru_use_laynorm", strtobool)
        self.ligru_use_laynorm_inp = strtobool(o["ligru_use_laynorm_inp"])
        self.ligru_use_batchnorm_inp = strtobool(o["ligru_use_batchnorm_inp"])
        self.ligru_orthinit = strtobool(o["ligru_orthinit"])
        self.ligru_act = _lst(o, "ligru_act")
        self.bidir = strtobool(o["ligru_bidir"])
        self.to_do = o.get("to_do", "train")
        self.prune = False
        self.guided_hcgs = False
        self.apply_guided_hcgs = False
        self.if_pattern = False
        self.skip_regularization = strtobool(o.get("skip_regularization", "False"))
        # pkc extension for config C3: the reference liGRU has no CGS hook; with
        # ligru_hcgs the LSTM's HCGS hook is reused (same keys hcgsx_* / hcgsh_*, masks drawn
        # after each layer's W and U Linears, applied in place every forward)
        self.ligru_hcgs = strtobool(o.get("ligru_hcgs", "False"))
        if self.ligru_hcgs:
            self.hcgsx_block = _lst(o, "hcgsx_block", int)
            self.hcgsh_block = _lst(o, "hcgsh_block", int)
            self.hcgsx_sparse = _lst(o, "hcgsx_sparse", float)
            self.hcgsh_sparse = _lst(o, "hcgsh_sparse", float)
            self.hcgsx, self.hcgsh = nn.ModuleList(), nn.ModuleList()
        self.wh, self.uh = nn.ModuleList(), nn.ModuleList()
        self.wz, self.uz = nn.ModuleList(), nn.ModuleList()
        self.ln, self.bn_wh, self.bn_wz = nn.ModuleList(), nn.ModuleList(), nn.ModuleList()
        if self.ligru_use_laynorm_inp:
            self.ln0 = LayerNorm(inp_dim)
        if self.ligru_use_batchnorm_inp:
            self.bn0 = nn.BatchNorm1d(inp_dim, momentum=0.05)
        cur = inp_dim
        for i, n in enumerate(self.ligru_lay):
            add_bias = not (self.ligru_use_laynorm[i] or self.ligru_use_batchnorm[i])
            self.wh.append(nn.Linear(cur, n, bias=add_bias))
            self.wz.append(nn.Linear(cur, n, bias=add_bias))
            if self.ligru_hcgs:
                self.hcgsx.append(_Mask(hcgs_mask(n, cur, self.hcgsx_block, self.hcgsx_sparse)))
            self.uh.append(nn.Linear(n, n, bias=False))
            self.uz.append(nn.Linear(n, n, bias=False))
            if self.ligru_hcgs:
                self.hcgsh.append(_Mask(hcgs_mask(n, n, self.hcgsh_block, self.hcgsh_sparse)))
            if self.ligru_orthinit:
                nn.init.orthogonal_(self.uh[i].weight)
                nn.init.orthogonal_(self.uz[i].weight)
            self.bn_wh.append(nn.BatchNorm1d(n, momentum=0.05))
            self.bn_wz.append(nn.BatchNorm1d(n, momentum=0.05))
            self.ln.append(LayerNorm(n))
            cur = 2 * n if self.bidir else n
        self.out_dim = cur

    def prune_parameters(self):
        raise NotImplementedError("the reference liGRU has no prune hook")

    def forward(self, x):
        """(T, B, F) -> (T, B, out_dim) on the pkc kernels (the shared-weight bidirectional
        convention when bidir), trainable under autograd (pkc.plugin)."""
        return arch_forward(self, x)

    def check_supported(self):
        pass

    def input_norm_specs(self):
        return _input_norm_specs(self, self.ligru_use_laynorm_inp, self.ligru_use_batchnorm_inp)

    def layer_specs(self):
        specs = []
        for i, n in enumerate(self.ligru_lay):
            specs.append(dict(H=n, act=self.ligru_act[i], bn=bool(self.ligru_use_batchnorm[i]),
                              drop=self.ligru_drop[i], bidir=bool(self.bidir),
                              W=[self.wz[i].weight, self.wh[i].weight],
                              b=[self.wz[i].bias, self.wh[i].bias],
                              U=[self.uz[i].weight, self.uh[i].weight],
                              bnm=[self.bn_wz[i], self.bn_wh[i]],
                              Wmask=self.hcgsx[i].mask if self.ligru_hcgs else None,
                              Umask=self.hcgsh[i].mask if self.ligru_hcgs else None,
                              ln=bool(self.ligru_use_laynorm[i]), ln_gamma=self.ln[i].gamma,
                              ln_beta=self.ln[i].beta))
        return specs


class GRU(nn.Module):
    """neural_networks.py:1240-1426 (options per proto/GRU.proto).  Parameters: wh, uh, wz, uz, wr,
    ur, ln, bn_wh, bn_wz, bn_wr (registration order and init draws of the reference)."""

    seq_model = True
    cell = "gru"
    GATES = ("z", "r", "h")

    def __init__(self, options, inp_dim):
        super().__init__()
        o = options
        self.input_dim = inp_dim
        self.gru_lay = _lst(o, "gru_lay", int)
        self.gru_drop = _lst(o, "gru_drop", float)
        self.gru_use_batchnorm = _lst(o, "gru_use_batchnorm", strtobool)
        self.gru_use_laynorm = _lst(o, "gru_use_laynorm", strtobool)
        self.gru_use_laynorm_inp = strtobool(o["gru_use_laynorm_inp"])
        self.gru_use_batchnorm_inp = strtobool(o["gru_use_batchnorm_inp"])
        self.gru_orthinit = strtobool(o["gru_orthinit"])
        self.gru_act = _lst(o, "gru_act")
        self.bidir = strtobool(o["gru_bidir"])
        self.to_do = o.get("to_do", "train")
        # core.run_nn / utils read these on every architecture; the reference GRU has no CGS hooks
        self.prune = False
        self.guided_hcgs = False
        self.apply_guided_hcgs = False
        self.if_pattern = False
        self.skip_regularization = strtobool(o.get("skip_regularization", "False"))
        self.wh, self.uh = nn.ModuleList(), nn.ModuleList()
        self.wz, self.uz = nn.ModuleList(), nn.ModuleList()
        self.wr, self.ur = nn.ModuleList(), nn.ModuleList()
        self.ln = nn.ModuleList()
        self.bn_wh, self.bn_wz, self.bn_wr = nn.ModuleList(), nn.ModuleList(), nn.ModuleList()
        if self.gru_use_laynorm_inp:
            self.ln0 = LayerNorm(inp_dim)
        if self.gru_use_batchnorm_inp:
            self.bn0 = nn.BatchNorm1d(inp_dim, momentum=0.05)
        cur = inp_dim
        for i, n in enumerate(self.gru_lay):
            add_bias = not (self.gru_use_laynorm[i] or self.gru_use_batchnorm[i])
            self.wh.append(nn.Linear(cur, n, bias=add_bias))
            self.wz.append(nn.Linear(cur, n, bias=add_bias))
            self.wr.append(nn.Linear(cur, n, bias=add_bias))
            self.uh.append(nn.Linear(n, n, bias=False))
            self.uz.append(nn.Linear(n, n, bias=False))
            self.ur.append(nn.Linear(n, n, bias=False))
            if self.gru_orthinit:
                nn.init.orthogonal_(self.uh[i].weight)
                nn.init.orthogonal_(self.uz[i].weight)
                nn.init.orthogonal_(self.ur[i].weight)
            self.bn_wh.append(nn.BatchNorm1d(n, momentum=0.05))
            self.bn_wz.append(nn.BatchNorm1d(n, momentum=0.05))
            self.bn_wr.append(nn.BatchNorm1d(n, momentum=0.05))
            self.ln.append(LayerNorm(n))
            cur = 2 * n if self.bidir else n
        self.out_dim = cur

    def prune_parameters(self):
        raise NotImplementedError("the reference GRU has no prune hook")

    def forward(self, x):
        """(T, B, F) -> (T, B, out_dim) on the pkc kernels (the shared-weight bidirectional
        convention when bidir), trainable under autograd (pkc.plugin)."""
        return arch_forward(self, x)

    def check_supported(self):
        pass

    def input_norm_specs(self):
        return _input_norm_specs(self, self.gru_use_laynorm_inp, self.gru_use_batchnorm_inp)

    def layer_specs(self):
        specs = []
        for i, n in enumerate(self.gru_lay):
            specs.append(dict(H=n, act=self.gru_act[i], bn=bool(self.gru_use_batchnorm[i]),
                              drop=self.gru_drop[i], bidir=bool(self.bidir),
                              W=[self.wz[i].weight, self.wr[i].weight, self.wh[i].weight],
                              b=[self.wz[i].bias, self.wr[i].bias, self.wh[i].bias],
                              U=[self.uz[i].weight, self.ur[i].weight, self.uh[i].weight],
                              bnm=[self.bn_wz[i], self.bn_wr[i], self.bn_wh[i]],
                              Wmask=None, Umask=None, ln=bool(self.gru_use_laynorm[i]),
                              ln_gamma=self.ln[i].gamma, ln_beta=self.ln[i].beta))
        return specs


class _PlainRec(nn.Module):
    """Shared construction of the reference's hook-free recurrent families (minimalGRU, RNN):
    option keys <prefix>_lay/_drop/_use_batchnorm/..., input Linears w<g> (bias only without
    BN/LN), recurrent Linears u<g> (no bias, optional orthogonal init), bn_w<g>, ln."""

    seq_model = True
    PREFIX = ""
    GATES = ()
    INIT_ORDER = ()         # reference registration / init order of the gate letters

    def __init__(self, options, inp_dim):
        super().__init__()
        o, p = options, self.PREFIX
        self.input_dim = inp_dim
        self.lay = _lst(o, p + "_lay", int)
        self.drop = _lst(o, p + "_drop", float)
        self.use_bn = _lst(o, p + "_use_batchnorm", strtobool)
        self.use_ln = _lst(o, p + "_use_laynorm", strtobool)
        self.ln_inp = strtobool(o[p + "_use_laynorm_inp"])
        self.bn_inp = strtobool(o[p + "_use_batchnorm_inp"])
        self.orthinit = strtobool(o[p + "_orthinit"])
        self.acts = _lst(o, p + "_act")
        self.bidir = strtobool(o[p + "_bidir"])
        self.to_do = o.get("to_do", "train")
        self.prune = False
        self.guided_hcgs = False
        self.apply_guided_hcgs = False
        self.if_pattern = False
        self.skip_regularization = strtobool(o.get("skip_regularization", "False"))
        for g in self.INIT_ORDER:
            setattr(self, "w" + g, nn.ModuleList())
            setattr(self, "u" + g, nn.ModuleList())
        self.ln = nn.ModuleList()
        for g in self.INIT_ORDER:
            setattr(self, "bn_w" + g, nn.ModuleList())
        if self.ln_inp:
            self.ln0 = LayerNorm(inp_dim)
        if self.bn_inp:
            self.bn0 = nn.BatchNorm1d(inp_dim, momentum=0.05)
        cur = inp_dim
        for i, n in enumerate(self.lay):
            add_bias = not (self.use_ln[i] or self.use_bn[i])
            for g in self.INIT_ORDER:
                getattr(self, "w" + g).append(nn.Linear(cur, n, bias=add_bias))
            for g in self.INIT_ORDER:
                getattr(self, "u" + g).append(nn.Linear(n, n, bias=False))
            if self.orthinit:
                for g in self.INIT_ORDER:
                    nn.init.orthogonal_(getattr(self, "u" + g)[i].weight)
            for g in self.INIT_ORDER:
                getattr(self, "bn_w" + g).append(nn.BatchNorm1d(n, momentum=0.05))
            self.ln.append(LayerNorm(n))
            cur = 2 * n if self.bidir else n
        self.out_dim = cur

    def prune_parameters(self):
        raise NotImplementedError("the reference %s has no prune hook" % type(self).__name__)

    def forward(self, x):
        """(T, B, F) -> (T, B, out_dim) on the pkc kernels (the shared-weight bidirectional
        convention when bidir), trainable under autograd (pkc.plugin)."""
        return arch_forward(self, x)

    def check_supported(self):
        pass

    def input_norm_specs(self):
        return _input_norm_specs(self, self.ln_inp, self.bn_inp)

    def layer_specs(self):
        specs = []
        for i, n in enumerate(self.lay):
            specs.append(dict(H=n, act=self.acts[i], bn=bool(self.use_bn[i]), drop=self.drop[i],
                              bidir=bool(self.bidir),
                              W=[getattr(self, "w" + g)[i].weight for g in self.GATES],
                              b=[getattr(self, "w" + g)[i].bias for g in self.GATES],
                              U=[getattr(self, "u" + g)[i].weight for g in self.GATES],
                              bnm=[getattr(self, "bn_w" + g)[i] for g in self.GATES],
                              Wmask=None, Umask=None, ln=bool(self.use_ln[i]),
                              ln_gamma=self.ln[i].gamma, ln_beta=self.ln[i].beta))
        return specs


class minimalGRU(_PlainRec):
    """neural_networks.py:1602-1777: z = sig(wz + Uz h); h = z h + (1-z) act(wh + Uh (z*h))*drop.
    Reference attribute names (minimalgru_lay, ...) are aliased below."""

    PREFIX = "minimalgru"
    cell = "minimalgru"
    GATES = ("z", "h")
    INIT_ORDER = ("h", "z")

    def __init__(self, options, inp_dim):
        super().__init__(options, inp_dim)
        self.minimalgru_lay, self.minimalgru_drop = self.lay, self.drop


class RNN(_PlainRec):
    """neural_networks.py:1780-1931: h = act(wh + Uh h) * drop."""

    PREFIX = "rnn"
    cell = "rnn"
    GATES = ("h",)
    INIT_ORDER = ("h",)

    def __init__(self, options, inp_dim):
        super().__init__(options, inp_dim)
        self.rnn_lay, self.rnn_drop = self.lay, self.drop


class LSTM(_PatternSet, nn.Module):
    """neural_networks.py:468-1237.  The reference forces bidir off inside forward (:835), so a
    bidirectional cfg crashes there on layer 2; pkc runs bidirectional LSTMs with the liGRU
    shared-weight convention (BASELINE C4) and uni-directional ones exactly as the reference."""

    seq_model = True
    cell = "lstm"
    GATES = ("f", "i", "o", "c")

    def __init__(self, options, inp_dim):
        super().__init__()
        o = options
        self.input_dim = inp_dim
        self.lstm_lay = _lst(o, "lstm_lay", int)
        self.lstm_drop = _lst(o, "lstm_drop", float)
        self.lstm_use_batchnorm = _lst(o, "lstm_use_batchnorm", strtobool)
        self.lstm_use_laynorm = _lst(o, "lstm_use_laynorm", strtobool)
        self.lstm_use_laynorm_inp = strtobool(o["lstm_use_laynorm_inp"])
        self.lstm_use_batchnorm_inp = strtobool(o["lstm_use_batchnorm_inp"])
        self.lstm_act = _lst(o, "lstm_act")
        self.lstm_orthinit = strtobool(o["lstm_orthinit"])
        self.bidir = strtobool(o["lstm_bidir"])
        self.to_do = o.get("to_do", "train")
        self.lstm_hcgs = strtobool(o.get("lstm_hcgs", "False"))
        self.hcgsx_block = _lst(o, "hcgsx_block", int) if "hcgsx_block" in o else []
        self.hcgsh_block = _lst(o, "hcgsh_block", int) if "hcgsh_block" in o else []
        self.hcgsx_sparse = _lst(o, "hcgsx_sparse", float) if "hcgsx_sparse" in o else []
        self.hcgsh_sparse = _lst(o, "hcgsh_sparse", float) if "hcgsh_sparse" in o else []
        self.lstm_quant = strtobool(o.get("lstm_quant", "False"))
        self.param_quant = _lst(o, "param_quant", int) if "param_quant" in o else [8] * len(self.lstm_lay)
        self.lstm_quant_inp = strtobool(o.get("lstm_quant_inp", "False"))
        self.inp_quant = _lst(o, "inp_quant", int) if "inp_quant" in o else [16]
        self.prune = strtobool(o.get("lstm_prune", "False"))
        self.prune_perc = _lst(o, "lstm_prune_perc", float) if "lstm_prune_perc" in o else [0.0]
        self.skip_regularization = strtobool(o.get("skip_regularization", "False"))
        self.guided_hcgs = strtobool(o.get("guided_hcgs", "False"))
        self.apply_guided_hcgs = strtobool(o.get("apply_guided_hcgs", "False"))
        self._pattern_opts(o)
        self.arch_name = o.get("arch_name", "LSTM")
        if self.lstm_hcgs:                      # registered first, as neural_networks.py:548-550
            self.hcgsx, self.hcgsh = nn.ModuleList(), nn.ModuleList()
        if self.guided_hcgs:                    # then the guided lists (553-564)
            for g in self.GATES:
                setattr(self, "ghcgs_w%sx" % g, nn.ModuleList())
                setattr(self, "ghcgs_u%sh" % g, nn.ModuleList())
        if self.if_pattern:
            self.pattern = {k: [] for k in ("pattern_w%sx" % g for g in self.GATES)}
            self.pattern.update({k: [] for k in ("pattern_u%sh" % g for g in self.GATES)})
            self.pattern_mask = {k: [] for k in ("pattern_mask_w%sx" % g for g in self.GATES)}
            self.pattern_mask.update({k: [] for k in ("pattern_mask_u%sh" % g for g in self.GATES)})
        for g in self.GATES:
            setattr(self, "w%sx" % g, nn.ModuleList())
            setattr(self, "u%sh" % g, nn.ModuleList())
        # registration order above = the reference's wfx, ufh, wix, uih, wox, uoh, wcx, uch
        # (neural_networks.py:606-616), so parameters() / optimizer indices line up
        self.ln = nn.ModuleList()
        for g in self.GATES:
            setattr(self, "bn_w%sx" % g, nn.ModuleList())
        if self.lstm_use_laynorm_inp:
            self.ln0 = LayerNorm(inp_dim)
        if self.lstm_use_batchnorm_inp:
            self.bn0 = nn.BatchNorm1d(inp_dim, momentum=0.05)
        cur = inp_dim
        for i, n in enumerate(self.lstm_lay):
            if not (self.lstm_use_laynorm[i] or self.lstm_use_batchnorm[i]):
                raise IndexError("the reference LSTM creates its W/U layers only with BN or LN "
                                 "(neural_networks.py:681-791)")
            for g in self.GATES:
                if self.lstm_quant:
                    lin = _QLinear(cur, n, self.param_quant[i], False,
                                   self.inp_quant[0] if self.lstm_quant_inp else None)
                else:
                    lin = nn.Linear(cur, n, bias=False)
                getattr(self, "w%sx" % g).append(lin)
            if self.lstm_hcgs:
                self.hcgsx.append(_Mask(hcgs_mask(n, cur, self.hcgsx_block, self.hcgsx_sparse)))
            if self.guided_hcgs:                # from the initial W (neural_networks.py:727-735)
                for g in self.GATES:
                    getattr(self, "ghcgs_w%sx" % g).append(_Mask(guided_hcgs_mask(
                        n, cur, self.hcgsx_block, self.hcgsx_sparse,
                        getattr(self, "w%sx" % g)[i].weight.data)))
            for g in self.GATES:
                if self.lstm_quant:
                    lin = _QLinear(n, n, self.param_quant[i], False,
                                   self.inp_quant[0] if self.lstm_quant_inp else None)
                else:
                    lin = nn.Linear(n, n, bias=False)
                getattr(self, "u%sh" % g).append(lin)
            if self.lstm_hcgs:
                self.hcgsh.append(_Mask(hcgs_mask(n, n, self.hcgsh_block, self.hcgsh_sparse)))
            if self.lstm_orthinit:
                for g in self.GATES:
                    nn.init.orthogonal_(getattr(self, "u%sh" % g)[i].weight)
            if self.guided_hcgs:                # from the initial U (neural_networks.py:797-806)
                for g in self.GATES:
                    getattr(self, "ghcgs_u%sh" % g).append(_Mask(guided_hcgs_mask(
                        n, n, self.hcgsh_block, self.hcgsh_sparse,
                        getattr(self, "u%sh" % g)[i].weight.data)))
            for g in self.GATES:
                getattr(self, "bn_w%sx" % g).append(nn.BatchNorm1d(n, momentum=0.05))
            self.ln.append(LayerNorm(n))
            cur = 2 * n if self.bidir else n
        self.out_dim = cur

    def prune_parameters(self):
        """Chunk-end pruning (neural_networks.py:1114-1135): every gate W and U at prune_perc[0]."""
        _prune_params([getattr(self, "%s" % nm)[i].weight for i in range(len(self.lstm_lay))
                       for nm in ("wfx", "wix", "wox", "wcx", "ufh", "uih", "uoh", "uch")],
                      self.prune_perc[0])
        return 1

    def apply_ghcgs(self):
        """Chunk-end regeneration of the guided masks from the current W / U (neural_networks.py:
        1137-1160, core.py:298-300)."""
        cur = self.input_dim
        for i, n in enumerate(self.lstm_lay):
            for g in self.GATES:
                _set_mask(getattr(self, "ghcgs_w%sx" % g)[i], guided_hcgs_mask(
                    n, cur, self.hcgsx_block, self.hcgsx_sparse, getattr(self, "w%sx" % g)[i].weight.data))
                _set_mask(getattr(self, "ghcgs_u%sh" % g)[i], guided_hcgs_mask(
                    n, n, self.hcgsh_block, self.hcgsh_sparse, getattr(self, "u%sh" % g)[i].weight.data))
            cur = 2 * n if self.bidir else n
        return 1

    def _gmask(self, kind, g, i):
        """Masks multiplied into w<g>x[i] / u<g>h[i] before use: HCGS, then guided HCGS when
        applied (neural_networks.py:858-873, 980-994)."""
        h = (self.hcgsx if kind == "w" else self.hcgsh)[i].mask if self.lstm_hcgs else None
        gm = None
        if self.guided_hcgs and self.apply_guided_hcgs:
            nm = ("ghcgs_w%sx" if kind == "w" else "ghcgs_u%sh") % g
            gm = getattr(self, nm)[i].mask
        return _mask_product(h, gm)

    def input_norm_specs(self):
        return _input_norm_specs(self, self.lstm_use_laynorm_inp, self.lstm_use_batchnorm_inp)

    def forward(self, x):
        """(T, B, F) -> (T, B, out_dim) on the pkc kernels (the shared-weight bidirectional
        convention when bidir), trainable under autograd (pkc.plugin)."""
        return arch_forward(self, x)

    def check_supported(self):
        if self.if_pattern and self.pattern_kernels is None and not self.can_search_patterns():
            raise NotImplementedError("pattern LSTM needs a pattern set (pattern_file option, "
                                      "patterns injected by run_nn) or pattern_num / pattern_nnz "
                                      "for the KMeans search")

    def pattern_params(self):
        """[(store key, layer, W or U, HCGS mask)] in the reference's update_mask order
        (neural_networks.py:1202-1223)."""
        out = []
        for i in range(len(self.lstm_lay)):
            for kind in ("w", "u"):
                for g in self.GATES:
                    nm = ("w%sx" if kind == "w" else "u%sh") % g
                    out.append((("pattern_mask_" + nm, i), i, getattr(self, nm)[i].weight,
                                self._gmask(kind, g, i)))
        return out

    def layer_specs(self):
        specs = []
        for i, n in enumerate(self.lstm_lay):
            specs.append(dict(H=n, act=self.lstm_act[i], bn=bool(self.lstm_use_batchnorm[i]),
                              drop=self.lstm_drop[i], bidir=bool(self.bidir),
                              W=[getattr(self, "w%sx" % g)[i].weight for g in self.GATES],
                              b=[None] * 4,
                              U=[getattr(self, "u%sh" % g)[i].weight for g in self.GATES],
                              bnm=[getattr(self, "bn_w%sx" % g)[i] for g in self.GATES],
                              Wmask=self.hcgsx[i].mask if self.lstm_hcgs else None,
                              Umask=self.hcgsh[i].mask if self.lstm_hcgs else None,
                              Wmasks=[self._gmask("w", g, i) for g in self.GATES],
                              Umasks=[self._gmask("u", g, i) for g in self.GATES],
                              qbits=self.param_quant[i] if self.lstm_quant else 0,
                              ibits=self.inp_quant[0] if (self.lstm_quant and self.lstm_quant_inp) else 0,
                              prune=self.prune_perc[i] if self.prune else None,
                              pattern=bool(self.if_pattern), ln=bool(self.lstm_use_laynorm[i]),
                              ln_gamma=self.ln[i].gamma, ln_beta=self.ln[i].beta))
        return specs
