"""Build libpkc.so (HIP kernels for gfx950 + the C ABI) in-tree with hipcc.

No cmake / no JIT cache: objects go to pytorch-kaldi-cgs_amd/build/, the shared library to
pytorch-kaldi-cgs_amd/pkc/libpkc.so so it travels with the repository snapshot to the GPU box.
"""
import concurrent.futures as cf
import glob
import hashlib
import os
import re
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
TOP = os.path.dirname(PKG)
CSRC = os.path.join(TOP, "csrc")
BUILD = os.path.join(TOP, "build")
LIB = os.path.join(PKG, "libpkc.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PKC_ARCH", "gfx950")
FLAGS = ["-O3", "-fPIC", "-std=c++17", "--offload-arch=" + ARCH, "-Wno-unused-result"]


INCLUDE = os.path.join(os.path.dirname(TOP), "include")


def src_digest(csrc=CSRC, include=INCLUDE):
    """SHA-256 over every file of csrc/ and include/ (relative name + bytes, sorted): embedded in
    libpkc.so at link time (pkc_src_digest) and recomputed by pkc._lib at load, so the library a
    process runs is tied to the sources of the tree it runs from."""
    h = hashlib.sha256()
    for root in (csrc, include):
        for f in sorted(os.listdir(root)):
            p = os.path.join(root, f)
            if os.path.isfile(p) and not f.startswith("."):
                h.update(("%s/%s\0" % (os.path.basename(root), f)).encode())
                with open(p, "rb") as fh:
                    h.update(fh.read())
                h.update(b"\0")
    return h.hexdigest()


def _digest_obj(digest):
    """build/pkc_digest.o: the one symbol carrying the source digest (regenerated when it moves)."""
    src = os.path.join(BUILD, "pkc_digest.cpp")
    obj = src + ".o"
    text = ('extern "C" const char* pkc_src_digest(void) { return "%s"; }\n' % digest)
    if not (os.path.exists(src) and open(src).read() == text and os.path.exists(obj)):
        with open(src, "w") as f:
            f.write(text)
        r = subprocess.run([HIPCC, "-O2", "-fPIC", "-x", "c++", "-c", src, "-o", obj],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed on %s:\n%s" % (src, r.stderr[-3000:]))
    return obj


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _deps(src, seen=None):
    """Headers `src` includes with "..." (recursively): a kernel file is rebuilt only when one of
    ITS headers changes (pkc_rnn.hip alone takes minutes)."""
    seen = set() if seen is None else seen
    for line in open(src):
        m = re.match(r'\s*#\s*include\s+"([^"]+)"', line)
        if m:
            h = os.path.normpath(os.path.join(os.path.dirname(src), m.group(1)))
            if os.path.exists(h) and h not in seen:
                seen.add(h)
                _deps(h, seen)
    return seen


def _compile(src, bdir=BUILD, defs=()):
    obj = os.path.join(bdir, os.path.basename(src) + ".o")
    newest_dep = max([os.path.getmtime(src)] + [os.path.getmtime(d) for d in _deps(src)])
    if os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj
    cmd = [HIPCC] + FLAGS + list(defs) + ["-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-O3", "-fPIC", "-std=c++17", "-x", "c++", "-c",
               src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed on %s:\n%s" % (src, r.stderr[-6000:]))
    return obj


# The phase-trace variant (measurement only, never the product): every source built with
# -DPKC_TRACE into build_trace/ and pkc/libpkc_trace.so, loaded with PKC_LIB=...; the step kernels
# then record s_memtime stamps per workgroup at their phase boundaries (pkc_rnn_impl.h PKC_TR)
TRACE_BUILD = os.path.join(TOP, "build_trace")
TRACE_LIB = os.path.join(PKG, "libpkc_trace.so")


def build(verbose=False, trace=False):
    bdir, lib = (TRACE_BUILD, TRACE_LIB) if trace else (BUILD, LIB)
    os.makedirs(bdir, exist_ok=True)
    srcs = _sources()
    defs = ("-DPKC_TRACE",) if trace else ()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, bdir, defs), srcs))
    digest = src_digest()
    objs.append(_digest_obj(digest))
    stamp = os.path.join(bdir, "libpkc.objs")
    listing = "\n".join(objs + [digest])
    same = os.path.exists(stamp) and open(stamp).read() == listing
    if same and os.path.exists(lib) and os.path.getmtime(lib) >= max(os.path.getmtime(o) for o in objs):
        return lib
    # RCCL: the pkc_dp_* all-reduce entry points for non-Python hosts
    cmd = [HIPCC, "-shared", "--offload-arch=" + ARCH, "-o", lib] + objs + [
        "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n%s" % r.stderr[-6000:])
    with open(stamp, "w") as f:            # a removed source also forces the next relink
        f.write(listing)
    if verbose:
        print("built", lib)
    return lib


if __name__ == "__main__":
    build(verbose=True, trace="--trace" in sys.argv)
    sys.exit(0)
