"""Zero-edit drop-in for the reference's `core` module.

run_exp.py resolves its training loop with `importlib.import_module('core')` and
`getattr(module, cfg['exp']['run_nn_script'])` (run_exp.py:81-83), and every shipped cfg names
`run_nn_script = run_nn`.  With this directory ahead of the reference checkout on PYTHONPATH,

    PYTHONPATH=<pkc>/pytorch-kaldi-cgs_amd/dropin:<pkc>/pytorch-kaldi-cgs_amd:<reference> \\
        python run_exp.py cfg/TIMIT_baselines/TIMIT_MLP_fmllr.cfg

`import core` lands here: the reference's own core.py (the next one on sys.path) is loaded under
the name `_reference_core` and every name it defines is re-exported, then `run_nn` is replaced by
pkc.core.run_nn (same signature, return value and side files, core.py:24-25, 362).  Neither the
reference's files nor its cfgs change; `arch_library = neural_networks` sections resolve to the
pkc classes inside pkc.core.run_nn.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_HERE = _os.path.dirname(_os.path.abspath(__file__))


def _reference_core():
    for d in _sys.path:
        d = _os.path.abspath(d or ".")
        f = _os.path.join(d, "core.py")
        if d != _HERE and _os.path.isfile(f):
            if "_reference_core" in _sys.modules:
                return _sys.modules["_reference_core"]
            spec = _ilu.spec_from_file_location("_reference_core", f)
            mod = _ilu.module_from_spec(spec)
            _sys.modules["_reference_core"] = mod
            spec.loader.exec_module(mod)
            return mod
    return None


_ref = _reference_core()
if _ref is not None:
    globals().update({k: v for k, v in vars(_ref).items() if not k.startswith("__")})

from pkc.core import run_nn  # noqa: E402,F401  (the pkc hot path replaces the reference's)
