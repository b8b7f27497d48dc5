"""Build the native libraries in-tree.

* ``libtmog_host.so`` -- C++17/OpenMP host kernels (CPU reference path of every device kernel,
  string hashing, tokenizer helpers). Built with ``g++``.
* ``libtmog_hip.so``  -- hand-written HIP kernels for CDNA4, ``hipcc --offload-arch=gfx950``.

Both are plain shared objects with a C ABI loaded through :mod:`ctypes`; they are compiled into
``transmogrifai_amd/ops/lib`` so the built objects travel with the repository snapshot.
"""
from __future__ import annotations

import fcntl
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
CSRC = ROOT / "csrc"
LIB = ROOT / "lib"
HOST_SO = LIB / "libtmog_host.so"
HIP_SO = LIB / "libtmog_hip.so"
ARCH = os.environ.get("TMOG_OFFLOAD_ARCH", "gfx950")


def _sources(kind: str):
    if kind == "host":
        return sorted((CSRC / "host").glob("*.cpp"))
    return sorted((CSRC / "hip").glob("*.hip"))


def _headers():
    return sorted(CSRC.rglob("*.h")) + sorted(CSRC.rglob("*.hpp")) + sorted(CSRC.rglob("*.inc"))


def _stale(so: Path, srcs) -> bool:
    if not so.exists():
        return True
    t = so.stat().st_mtime
    return any(s.stat().st_mtime > t for s in list(srcs) + _headers())


def hipcc_path():
    p = shutil.which("hipcc")
    if p:
        return p
    cand = "/opt/rocm/bin/hipcc"
    return cand if os.path.exists(cand) else None


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed ({' '.join(map(str, cmd))}):\n{r.stdout}")
    return r.stdout


class _Lock:
    def __enter__(self):
        LIB.mkdir(parents=True, exist_ok=True)
        self.f = open(LIB / ".build.lock", "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *a):
        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()


def build_host(force: bool = False) -> Path:
    srcs = _sources("host")
    with _Lock():
        if force or _stale(HOST_SO, srcs):
            tmp = HOST_SO.with_suffix(f".so.tmp{os.getpid()}")
            cxx = shutil.which("g++") or "c++"
            import sysconfig
            # utf8_pack.cpp reads str objects through the CPython API (symbols from the running interpreter)
            _run([cxx, "-O3", "-march=x86-64-v2", "-ffp-contract=off", "-std=c++17", "-fopenmp", "-fPIC", "-shared",
                  f"-I{CSRC}", f"-I{sysconfig.get_paths()['include']}", "-o", str(tmp)] + [str(s) for s in srcs])
            os.replace(tmp, HOST_SO)
    return HOST_SO


def build_hip(force: bool = False, arch: str = ARCH) -> Path:
    srcs = _sources("hip")
    hipcc = hipcc_path()
    if hipcc is None:
        raise RuntimeError("hipcc not found: cannot build the HIP kernels")
    with _Lock():
        if force or _stale(HIP_SO, srcs):
            from concurrent.futures import ThreadPoolExecutor
            objs = [str(LIB / (s.stem + ".o")) for s in srcs]
            # one hipcc per translation unit, a few at a time (the tree kernels alone take ~1 min)
            with ThreadPoolExecutor(max_workers=max(1, min(8, os.cpu_count() or 1))) as ex:
                list(ex.map(lambda so: _run([hipcc, f"--offload-arch={arch}", "-O3", "-std=c++17", "-fPIC", "-c",
                                             "-munsafe-fp-atomics", f"-I{CSRC}", "-o", so[1], str(so[0])]),
                            zip(srcs, objs)))
            tmp = HIP_SO.with_suffix(f".so.tmp{os.getpid()}")
            _run([hipcc, f"--offload-arch={arch}", "-shared", "-fPIC", "-o", str(tmp)] + objs + ["-lrccl"])
            os.replace(tmp, HIP_SO)
            for o in objs:
                try:
                    os.remove(o)
                except OSError:
                    pass
    return HIP_SO


def build_all(force: bool = False):
    build_host(force)
    build_hip(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print(HOST_SO, HIP_SO)
