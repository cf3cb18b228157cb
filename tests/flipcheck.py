"""Counted tolerances for comparisons that one element can move by a branch.

Two runs whose arithmetic differs only in rounding (summation order, or the GPU's compensated bf16
products against their CPU restatement) agree to ~1e-6 relative on every smooth quantity.  Two
mechanisms move single elements by much more, and both are counted here instead of being absorbed
into a loose norm bound:

* a ReLU pre-activation within rounding of 0 takes the other branch: that element's dz enters or
  leaves its BatchNorm column sums, which moves the column's whole gradient (pre-activation sign
  flips, counted per layer: sign_flips);
* RMSprop's first steps are lr * g / sqrt((1 - alpha) g^2) = +-4.47 lr whatever |g| is, so a
  gradient within rounding of zero whose sign differs moves its weight by ~9 lr (sign steps,
  counted per tensor: step_outliers).

A systematic defect moves a large share of the elements; these mechanisms move a handful.  The
assertions bound the COUNT (with the measured count in the message) and hold everything else at
the tight bound.
"""
import numpy as np
import torch


def sign_flips(a, b):
    """Elements of a and b (same shape) on different sides of zero."""
    a = torch.as_tensor(a).double().reshape(-1).cpu()
    b = torch.as_tensor(b).double().reshape(-1).cpu()
    return int(((a > 0) != (b > 0)).sum().item())


def step_outliers(got, ref, tol_rel, scale=None):
    """(count, max |diff|, max |diff| over the other elements / scale): elements of got differing from
    ref by more than tol_rel * scale (scale: max |ref| by default)."""
    g = torch.as_tensor(got).double().reshape(-1).cpu()
    r = torch.as_tensor(ref).double().reshape(-1).cpu()
    s = float(r.abs().max()) if scale is None else float(scale)
    s = max(s, 1e-30)
    d = (g - r).abs()
    out = d > tol_rel * s
    n = int(out.sum().item())
    rest = float(d[~out].max()) / s if bool((~out).any()) else 0.0
    return n, float(d.max()) if d.numel() else 0.0, rest


def assert_counted(name, n, size, frac, max_abs, bound_abs, detail=""):
    """At most frac of size (and at least one allowed) outliers, none beyond bound_abs."""
    allowed = max(1, int(frac * size))
    assert n <= allowed, "%s: %d of %d elements outside the tight bound (allowed %d) %s" % (
        name, n, size, allowed, detail)
    assert max_abs <= bound_abs, "%s: an element moved %.3g (> %.3g) %s" % (
        name, max_abs, bound_abs, detail)


def optim_state_by_name(sd, net, onet):
    """A torch.optim state_dict indexed over net.parameters(), re-indexed over onet.parameters()
    (the oracle class may register its parameters in another order); tensors to the CPU."""
    names = [n for n, _ in net.named_parameters()]
    where = {n: i for i, (n, _) in enumerate(onet.named_parameters())}
    state = {where[names[i]]: {a: (b.detach().cpu().clone() if torch.is_tensor(b) else b)
                               for a, b in st.items()} for i, st in sd["state"].items()}
    group = dict(sd["param_groups"][0])
    group["params"] = list(range(len(where)))
    return {"state": state, "param_groups": [group]}


def resync(nets, onets, opt_sds, oopts):
    """The oracle's starting state := the GPU side's (parameters, buffers, optimizer state), so a
    step is compared from a common start and one step's rounding flips do not compound."""
    for k in nets:
        onets[k].load_state_dict({n: v.detach().cpu().clone() for n, v in nets[k].state_dict().items()})
        if opt_sds is not None:
            oopts[k].load_state_dict(optim_state_by_name(opt_sds[k], nets[k], onets[k]))
