"""Oracle: ONE recurrent time step restated from a given state, for every step at once
(test infrastructure only — imported by tests/, never by the product path).

oracle.nets runs the reference's time loops end to end, so two implementations that differ in one
rounding at step t differ everywhere after it.  These functions instead take the state a run
actually had before each step (h_{t-1}, and in the BPTT the carried gradients' operands) and
restate that ONE step, vectorised over t: a per-time-step check of a GPU run's saved tensors in
which nothing compounds, so an error of the step kernels shows as itself and a summation-order
difference stays at fp32 rounding.

  liGRU  neural_networks.py:1576-1584   z = sig(wz + Uz h); hc = act(wh + Uh h) * m;
                                         h = z h + (1 - z) hc
  LSTM   neural_networks.py:1087-1092   f, i, o = sig(w. + U. h); c = i act(wc + Uc h) m + f c;
                                         h = o act(c)
The backward functions are the chain rule of those expressions (what autograd computes for the
reference's loop): the BPTT of step t from dL/dy_t, the products of step t+1's gate gradients with
U (dh_t = sum_g dgates_g,t+1 U_g) and the carried dL/dh (liGRU: g_{t+1} z_{t+1}) / dL/dc (LSTM:
dc_{t+1} f_{t+1}).  The carries are elementwise and contract (|z|, |f| < 1): they are recomputed
here from the given operands in float64 (steps_ligru_bwd / steps_lstm_bwd), only the product
operands are taken from the run.  Pinned against autograd of oracle.nets' loops by
tests/test_oracle_steps_cpu.py.

Layout: "processing time" (T, R, H) with R = B (uni) or 2B (the liGRU / C4 shared-weight
bidirectional convention: rows >= B run the reversed sequence, their step t reads input time
T - 1 - t) — the layout of pkc's saved hs / gates / dgates.
"""
import torch


def act_fwd(name, x):
    """neural_networks.py:54-78 (the activations a recurrent layer uses)."""
    if name == "relu":
        return torch.relu(x)
    if name == "tanh":
        return torch.tanh(x)
    if name == "sigmoid":
        return torch.sigmoid(x)
    if name in ("linear", "leaky_relu_1"):
        return x
    raise ValueError(name)


def act_bwd_out(name, y):
    """d act / d x expressed in the activation's OUTPUT y (what a saved post-activation allows)."""
    if name == "relu":
        return (y > 0).to(y.dtype)
    if name == "tanh":
        return 1 - y * y
    if name == "sigmoid":
        return y * (1 - y)
    if name == "linear":
        return torch.ones_like(y)
    raise ValueError(name)


def to_proc_time(x, B, bidir):
    """(T, B, H) tensor in input time -> (T, R, H) processing time: row r >= B of step t reads
    input time T - 1 - t (neural_networks.py:1536-1538 cat/flip)."""
    if not bidir:
        return x
    return torch.cat([x, torch.flip(x, [0])], 1)


def out_grad_proc_time(dy, B, H, bidir):
    """dL/dy (T, B, D) of a layer output y = cat(h_f, flip(h_b)) (neural_networks.py:1590-1594)
    -> dL/dh in processing time (T, R, H)."""
    if not bidir:
        return dy
    return torch.cat([dy[:, :, :H], torch.flip(dy[:, :, H:], [0])], 1)


def steps_ligru_fwd(hA, hprev, U, wpre, mask, act):
    """Every step t from its given h_{t-1}: hA (T, R, H) the operand the products read (h_{t-1}
    itself, or its bf16 copy in pkc's bf16 step mode), hprev (T, R, H) the h_{t-1} of the update,
    U = [Uz, Uh] (H, H) as the products read them, wpre = [wz, wh] (T, R, H) the (BatchNorm'd)
    input projections in processing time, mask (R, H) the recurrent dropout mask (NOT rescaled).
    Returns (z, act(a), h), each (T, R, H)."""
    z = torch.sigmoid(wpre[0] + hA @ U[0].t())
    hcr = act_fwd(act, wpre[1] + hA @ U[1].t())
    return z, hcr, z * hprev + (1 - z) * (hcr * mask)


def steps_lstm_fwd(hA, hprev, cprev, U, wpre, mask, act):
    """LSTM (neural_networks.py:1087-1092) from given h_{t-1} (hA: the products' operand, hprev
    unused but kept for symmetry) and c_{t-1}; U = [Uf, Ui, Uo, Uc], wpre likewise.  Returns
    (f, i, o, act(cand), c, h)."""
    f = torch.sigmoid(wpre[0] + hA @ U[0].t())
    i = torch.sigmoid(wpre[1] + hA @ U[1].t())
    o = torch.sigmoid(wpre[2] + hA @ U[2].t())
    cc = act_fwd(act, wpre[3] + hA @ U[3].t())
    c = i * cc * mask + f * cprev
    return f, i, o, cc, c, o * act_fwd(act, c)


def steps_ligru_bwd(dh_y, dgA, U, z, hcr, hprev, mask, act):
    """BPTT of the liGRU steps: dh_y (T, R, H) dL/dh_t from the layer output, dgA [dz, da] (T, R,
    H) the gate gradients of every step as the BPTT products read them (fp32, or their bf16
    copies), U = [Uz, Uh], z / hcr / hprev the forward's saved tensors.  The recurrent part of
    dL/dh_t is dgA_t+1 @ U (from the run's operands) + g_{t+1} z_{t+1} (this function's own
    carry).  Returns the gate gradients (dz_pre, da_pre) (T, R, H) and the g chain."""
    T = dh_y.shape[0]
    prod = torch.zeros_like(dh_y)
    prod[:-1] = dgA[0][1:] @ U[0] + dgA[1][1:] @ U[1]   # dh_t from step t + 1's products
    dz = torch.empty_like(dh_y)
    da = torch.empty_like(dh_y)
    gs = torch.empty_like(dh_y)
    g = None
    for t in range(T - 1, -1, -1):
        gt = dh_y[t] + prod[t] + (g * z[t + 1] if g is not None else 0)
        hc = hcr[t] * mask
        dz[t] = gt * (hprev[t] - hc) * z[t] * (1 - z[t])
        da[t] = gt * (1 - z[t]) * mask * act_bwd_out(act, hcr[t])
        gs[t] = g = gt
    return dz, da, gs


def steps_lstm_bwd(dh_y, dgA, U, f, i, o, cc, c, cprev, mask, act):
    """BPTT of the LSTM steps (gate order f, i, o, cand): the recurrent part of dL/dh_t is
    sum_g dgA_g,t+1 @ U_g; dL/dc_t = g o act'(act(c_t)) + dc_{t+1} f_{t+1} (own carry).  Returns
    the four pre-activation gradients (T, R, H)."""
    T = dh_y.shape[0]
    prod = torch.zeros_like(dh_y)
    prod[:-1] = sum(dgA[q][1:] @ U[q] for q in range(4))
    out = [torch.empty_like(dh_y) for _ in range(4)]
    carry = None
    for t in range(T - 1, -1, -1):
        g = dh_y[t] + prod[t]
        tc = act_fwd(act, c[t])
        dc = g * o[t] * act_bwd_out(act, tc) + (carry if carry is not None else 0)
        out[0][t] = dc * cprev[t] * f[t] * (1 - f[t])
        out[1][t] = dc * cc[t] * mask * i[t] * (1 - i[t])
        out[2][t] = g * tc * o[t] * (1 - o[t])
        out[3][t] = dc * i[t] * mask * act_bwd_out(act, cc[t])
        carry = dc * f[t]
    return out


def pre_grad_input_time(dg, B, bidir):
    """Gate gradients (T, R, H) -> dL/d(pre-activation rows) (T, B, H) in input time: the two
    directions read the same projection rows (shared W, neural_networks.py:1536-1538), so both
    contributions add."""
    if not bidir:
        return dg
    return dg[:, :B] + torch.flip(dg[:, B:], [0])


def weight_grad(dg, hA):
    """dU_g = sum_{t, r} dgates_g[t, r, :]^T h_{t-1}[r, :] (dg, hA (T, R, H))."""
    H = dg.shape[-1]
    return dg.reshape(-1, H).t() @ hA.reshape(-1, hA.shape[-1])
