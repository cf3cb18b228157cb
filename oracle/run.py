"""Oracle: the [model] DSL interpreter and one run_nn training/forward step (test only).

Restates utils.forward_model (utils.py:1884-2050) for the operations the hot path uses
(compute / cost_nll / cost_err / sum / mult_constant / concatenate) and the core.run_nn batch
body (core.py:216-232: forward, zero_grad, backward, step per architecture).
"""
import re

import torch

from .nets import nll_err

_PAT = re.compile(r"(.*)=(.*)\((.*),(.*)\)")


_PAT3 = re.compile(r"(.*)=(.*)\((.*),(.*),(.*)\)")


def parse_model(text):
    """utils.py:1898-1903: out=op(a,b) (greedy: the LAST comma splits); a line whose output name
    starts with 'loss_gl' is re-read as out=op(a,b,c) and c rides in b as "b,c"."""
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


def _reg_norm(nets, op, lam):
    """utils.py:24-60 (l1_norm / l2_norm / gl_norm) and the guided-HCGS zero (1954-1991)."""
    first = next(iter(nets.values()))
    if getattr(first, "apply_guided_hcgs", False):
        return torch.tensor(0.0)
    if op == "cost_gl":
        lam, nblk = lam.split(",")
    acc = torch.tensor(0.0, dtype=torch.float32)
    for net in nets.values():
        for p in net.parameters():
            if p.dim() > 1 and not net.skip_regularization:
                if op == "cost_l1":
                    acc = acc + torch.norm(p, 1)
                elif op == "cost_l2":
                    acc = acc + torch.norm(p, 2)
                else:
                    for d1 in torch.chunk(p, int(nblk), 1):
                        for blk in torch.chunk(d1, int(nblk), 0):
                            acc = acc + torch.norm(blk, 2)
    return acc * float(lam)


def forward_model(lines, nets, seq, fea_cols, lab_cols, inp, max_len=0, batch=0, forward_out=None):
    """utils.py:1884-2050.  seq: {arch: bool}; fea_cols: {fea: (c0, c1)}; lab_cols: {lab: col}."""
    outs = {}
    for fea, (c0, c1) in fea_cols.items():         # utils.py:1891-1896: input features first
        outs[fea] = inp[..., c0:c1]
    for out_name, op, a, b in lines:
        if op == "compute":
            if b in fea_cols:
                c0, c1 = fea_cols[b]
                x = inp[..., c0:c1]
                if x.dim() == 3 and not seq[a]:
                    x = x.reshape(max_len * batch, -1)
                if x.dim() == 2 and seq[a]:
                    x = x.view(max_len, batch, -1)
            else:
                x = outs[b]
                if not seq[a] and x.dim() == 3:
                    x = outs[b] = x.reshape(max_len * batch, -1)
                if seq[a] and x.dim() == 2:
                    x = outs[b] = x.view(max_len, batch, -1)
            outs[out_name] = nets[a](x)
            if forward_out is not None and out_name == forward_out:
                break
        elif op in ("cost_nll", "cost_err"):
            lab = inp[..., lab_cols[b]].reshape(-1)
            o = outs[a]
            if o.dim() == 3:
                o = o.reshape(-1, o.shape[-1])
            loss, err = nll_err(o, lab)
            outs[out_name] = loss if op == "cost_nll" else err
        elif op == "sum":
            outs[out_name] = outs[a] + outs[b]
        elif op == "mult_constant":
            outs[out_name] = outs[a] * float(b)
        elif op in ("cost_l1", "cost_l2", "cost_gl"):
            outs[out_name] = _reg_norm(nets, op, b)
        elif op == "concatenate":
            outs[out_name] = torch.cat((outs[a], outs[b]), outs[a].dim() - 1)
        else:
            raise NotImplementedError(op)
    return outs


def train_step(lines, nets, opts, seq, fea_cols, lab_cols, inp, max_len=0, batch=0):
    """core.py:216-232."""
    outs = forward_model(lines, nets, seq, fea_cols, lab_cols, inp, max_len, batch)
    for o in opts.values():
        o.zero_grad()
    outs["loss_final"].backward()
    for o in opts.values():
        o.step()
    return outs
