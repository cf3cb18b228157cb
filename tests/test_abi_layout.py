"""The ctypes mirrors in pkc._lib have the layout of the C structs in include/pkc.h: gcc compiles a
probe printing sizeof / offsetof of every field the Python side names (a field appended on one side
only — e.g. pkc_dense_bwd_args.dz_scratch — would shift nothing but the size, or everything after a
field inserted in the middle; both are caught).  CPU only: no GPU, no HIP."""
import ctypes as C
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))

PAIRS = [("DenseFwdArgs", "pkc_dense_fwd_args"), ("DenseBwdArgs", "pkc_dense_bwd_args"),
         ("NllArgs", "pkc_nll_args"), ("OptTensor", "pkc_opt_tensor"), ("RnnArgs", "pkc_rnn_args"),
         ("GemmProblem", "pkc_gemm_problem"), ("RegItem", "pkc_reg_item"), ("OptSeg", "pkc_opt_seg"),
         ("BnBwdEpi", "pkc_bn_bwd_epi")]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_ctypes_structs_match_header(tmp_path):
    from pkc import _lib as L
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "pkc.h"', "int main(void) {"]
    expect = []
    for py, cname in PAIRS:
        cls = getattr(L, py)
        lines.append('printf("%%zu\\n", sizeof(%s));' % cname)
        expect.append(("sizeof " + cname, C.sizeof(cls)))
        for f in cls._fields_:
            lines.append('printf("%%zu\\n", offsetof(%s, %s));' % (cname, f[0]))
            expect.append(("%s.%s" % (cname, f[0]), getattr(cls, f[0]).offset))
    lines += ["return 0;", "}"]
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True,
                                          text=True).stdout.split()]
    assert len(got) == len(expect)
    bad = [(k, v, g) for (k, v), g in zip(expect, got) if v != g]
    assert not bad, "ctypes vs C layout (name, ctypes, C): %s" % bad


# sha256 over the (field, offset) list + sizes of every mirrored struct, per PKC_ABI_VERSION: a
# struct that changes without a version bump fails here (bump PKC_ABI_VERSION in include/pkc.h and
# pkc._lib.ABI_VERSION, then record the new digest under the new version)
LAYOUT_DIGEST = {2: "aff881268bdfc4a5ffb16199eb028e3b1bdaaa98595e969dfe4d7a2fbfa09b47",
                 3: "29670d34ec50ca9c1650f053da10b2d570ed9bff4e9d0d22f31b11ca9c53e012",
                 4: "29670d34ec50ca9c1650f053da10b2d570ed9bff4e9d0d22f31b11ca9c53e012",
                 5: "2c453ea47366535096140ab754d5ecfcd019ccecde60defafc6b607b14f5eb2d",
                 6: "1bcf851b6b8c7c47b5d010bb84ad5bfed004e6061606a15f6e24fda230644bd9",
                 7: "e7c2d5119718927e74e47e4889727b8834bcec21da87a549b5a754e85736ecb5",
                 8: "9e28b5a7ec480789bbdddbba246843db7d0589d5f3d0eb7cc95c8c98bcc8cc2f",
                 9: "9e28b5a7ec480789bbdddbba246843db7d0589d5f3d0eb7cc95c8c98bcc8cc2f"}


def _layout_digest(L):
    import hashlib
    h = hashlib.sha256()
    for py, cname in PAIRS:
        cls = getattr(L, py)
        h.update(("%s %d;" % (cname, C.sizeof(cls))).encode())
        for f in cls._fields_:
            h.update(("%s@%d;" % (f[0], getattr(cls, f[0]).offset)).encode())
    return h.hexdigest()


def test_abi_version_matches_header_and_layout():
    import re
    from pkc import _lib as L
    hdr = open(os.path.join(ROOT, "include", "pkc.h")).read()
    v = int(re.search(r"#define PKC_ABI_VERSION (\d+)", hdr).group(1))
    assert v == L.ABI_VERSION
    assert v in LAYOUT_DIGEST, "PKC_ABI_VERSION %d has no recorded layout digest" % v
    assert _layout_digest(L) == LAYOUT_DIGEST[v], (
        "struct layout changed under PKC_ABI_VERSION %d: bump the version" % v)
