"""Which time-loop form pkc_rnn_fwd / pkc_rnn_bwd take for a layer (pkc_rnn_persist_form,
include/pkc.h: 1 the liGRU loops, 2 the grid-synchronised loops, 0 one launch per step) at the
BASELINE sequence configs' layer shapes, and where the rules fall back.  The function reads only
the argument struct and the environment (with no device it assumes 256 compute units), so the
dispatch rules are checked here without a GPU; tests/test_gpu_lstm_persist.py checks each loop
against the per-step launches on the GPU."""
import ctypes as C
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))


def _args(cell, H, B, bidir=False, **kw):
    """An RnnArgs with non-null placeholder pointers (never dereferenced by the form query)."""
    from pkc import _lib as L
    a = L.RnnArgs()
    a.cell, a.T, a.B, a.H, a.bidir = cell, 40, B, H, int(bidir)
    p = C.c_void_p(4096)
    for f in ("wpre", "hs", "cs", "gates", "y", "dy", "dgates", "work", "ut"):
        setattr(a, f, p)
    for g in range(4):
        a.U[g] = p
    for k, v in kw.items():
        if k == "U_h":
            for g in range(4):
                a.U_h[g] = p if v else None
        elif isinstance(v, bool):
            setattr(a, k, p if v else None)
        else:
            setattr(a, k, v)
    return a


def _form(a):
    from pkc import _lib as L
    lib = L.lib()
    return lib.pkc_rnn_persist_form(C.byref(a), 0), lib.pkc_rnn_persist_form(C.byref(a), 1)


def test_c4_lstm_fp32_and_bf16_take_the_grid_loops():
    from pkc import _lib as L
    # C4: 4 x 1024 bidirectional, B = 16 (32 rows)
    assert _form(_args(L.CELL_LSTM, 1024, 16, True)) == (2, 2)
    assert _form(_args(L.CELL_LSTM, 1024, 16, True, step_bf16=1, hs_h=True, U_h=True,
                       ut_h=True, dgates_h=True)) == (2, 2)
    assert _form(_args(L.CELL_LSTM, 512, 12, False)) == (2, 2)
    assert _form(_args(L.CELL_LSTM, 768, 10, True)) == (2, 2)


def test_c5_quantised_h_loops():
    from pkc import _lib as L
    q = dict(qbits=16, qh_exact=1, hq=True, U_h=True)
    assert _form(_args(L.CELL_LSTM, 512, 12, False, **q)) == (2, 2)
    # forward loops for H = 768 / 1024; their BPTT keeps the per-step launches (H = 512 only)
    assert _form(_args(L.CELL_LSTM, 1024, 16, False, **q)) == (2, 0)


def test_c3_ligru_fp32_grid_loops():
    from pkc import _lib as L
    assert _form(_args(L.CELL_LIGRU, 550, 8, True)) == (2, 2)     # C3: 16 rows
    assert _form(_args(L.CELL_LIGRU, 24, 4, False)) == (2, 2)
    assert _form(_args(L.CELL_LIGRU, 550, 9, True)) == (0, 0)     # 18 rows > 16
    assert _form(_args(L.CELL_LIGRU, 1024, 8, True)) == (0, 0)    # H > 768


@pytest.mark.parametrize("case", ["small_h", "too_many_rows", "layernorm", "block_sparse",
                                  "quant_not_exact", "gru"])
def test_per_step_fallbacks(case):
    from pkc import _lib as L
    a = {"small_h": lambda: _args(L.CELL_LSTM, 256, 16, True),
         "too_many_rows": lambda: _args(L.CELL_LSTM, 1024, 17, True),     # 34 rows > 32
         "layernorm": lambda: _args(L.CELL_LSTM, 1024, 16, True, ln_gamma=True),
         "block_sparse": lambda: _args(L.CELL_LSTM, 1024, 16, True, kmap_fwd=True, kmap_bwd=True),
         "quant_not_exact": lambda: _args(L.CELL_LSTM, 512, 12, False, qbits=16, hq=True),
         "gru": lambda: _args(L.CELL_GRU, 550, 8, True)}[case]()
    assert _form(a) == (0, 0)


def test_environment_switches(monkeypatch):
    from pkc import _lib as L
    monkeypatch.setenv("PKC_RNN_LSTM_F32", "0")          # the fp32 LSTM loops only
    assert _form(_args(L.CELL_LSTM, 1024, 16, True)) == (0, 0)
    assert _form(_args(L.CELL_LSTM, 1024, 16, True, step_bf16=1, hs_h=True, U_h=True,
                       ut_h=True, dgates_h=True)) == (2, 2)
    monkeypatch.setenv("PKC_RNN_LSTM_PERSIST", "0")      # every LSTM loop
    assert _form(_args(L.CELL_LSTM, 1024, 16, True, step_bf16=1, hs_h=True, U_h=True,
                       ut_h=True, dgates_h=True)) == (0, 0)
    monkeypatch.setenv("PKC_RNN_LIGRU_GRID", "0")
    assert _form(_args(L.CELL_LIGRU, 550, 8, True)) == (0, 0)
