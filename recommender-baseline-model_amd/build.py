"""Build librecsys_hip.so (the C-ABI hot-path library) for gfx950, in-tree.

    python recommender-baseline-model_amd/build.py [--force]

Compiles every ``csrc/*.hip`` with hipcc (``--offload-arch=gfx950``) into an
object file under ``csrc/build/`` and links them into
``recommender-baseline-model_amd/librecsys_hip.so``.  Incremental: a source is
rebuilt only when it (or a header) is newer than its object.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(CSRC, "build")
LIB = os.path.join(PKG, "librecsys_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RS_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         "-I", os.path.join(ROOT, "include"), "-I", CSRC]


def _headers_mtime():
    hs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _included(path):
    with open(path) as fh:
        return fh.readline().startswith("// rs-build: included")


def _included_mtime():
    inc = [p for p in glob.glob(os.path.join(CSRC, "*.hip")) if _included(p)]
    return max((os.path.getmtime(p) for p in inc), default=0.0)


def _compile(src, force):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj):
        if os.path.getmtime(obj) >= max(os.path.getmtime(src), _headers_mtime(), _included_mtime()):
            return obj, False
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj, True


def build(force=False, jobs=None):
    os.makedirs(OBJ, exist_ok=True)
    # sources marked "rs-build: included" on line 1 are compiled inside the file that includes them
    srcs = [p for p in sorted(glob.glob(os.path.join(CSRC, "*.hip"))) if not _included(p)]
    jobs = jobs or min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force), srcs))
    objs = [o for o, _ in results]
    rebuilt = any(b for _, b in results)
    if rebuilt or force or not os.path.exists(LIB) or \
            os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
