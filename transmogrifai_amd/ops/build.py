"""Build the native libraries in-tree.

* ``libtmog_host.so`` -- C++17/OpenMP host kernels (CPU reference path of every device kernel,
  string hashing, tokenizer helpers). Built with ``g++``.
* ``libtmog_hip.so``  -- hand-written HIP kernels for CDNA4, ``hipcc --offload-arch=gfx950``.

Both are plain shared objects with a C ABI loaded through :mod:`ctypes`; they are compiled into
``transmogrifai_amd/ops/lib`` so the built objects travel with the repository snapshot.

Provenance: each library embeds ``TMOG_SRC_HASH=<sha256>`` -- the hash of the sources, headers and compile flags
it was built from (:func:`source_hash`). A library is stale when its embedded hash differs from the tree's
(modification times are not trusted: a snapshot copy resets them), and :mod:`._native` refuses to load a library
whose hash does not match the sources next to it.
"""
from __future__ import annotations

import fcntl
import hashlib
import os
import re
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


HOST_FLAGS = ["-O3", "-march=x86-64-v2", "-ffp-contract=off", "-std=c++17", "-fopenmp", "-fPIC", "-shared"]
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-c", "-munsafe-fp-atomics"]
_HASH_RE = re.compile(rb"TMOG_SRC_HASH=([0-9a-f]{64})")


def source_hash(kind: str, arch: str = ARCH) -> str:
    """sha256 over the library's sources, every header and the compile flags (the library's identity)."""
    h = hashlib.sha256()
    flags = HOST_FLAGS if kind == "host" else HIP_FLAGS + [f"--offload-arch={arch}"]
    h.update(" ".join([kind] + flags).encode())
    for f in list(_sources(kind)) + _headers():
        h.update(b"\0" + str(f.relative_to(CSRC)).encode() + b"\0")
        h.update(f.read_bytes())
    return h.hexdigest()


def embedded_hash(so: Path):
    """The source hash a built library carries, or None (not built / built without provenance)."""
    try:
        m = _HASH_RE.search(Path(so).read_bytes())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _stale(so: Path, kind: str) -> bool:
    return embedded_hash(so) != source_hash(kind)


def _provenance_source(kind: str, digest: str) -> Path:
    """A translation unit holding the hash as data (found by :func:`embedded_hash`) and behind an accessor."""
    LIB.mkdir(parents=True, exist_ok=True)
    src = LIB / (f"provenance_{kind}." + ("cpp" if kind == "host" else "hip"))
    src.write_text(f'extern "C" __attribute__((used)) const char tmog_{kind}_src_hash[] = "TMOG_SRC_HASH={digest}";\n'
                   f'extern "C" const char* tmog_{kind}_source_hash() {{ return tmog_{kind}_src_hash + 14; }}\n')
    return src


def verify(so: Path, kind: str) -> None:
    """Raise if ``so`` was not built from the sources in this tree."""
    got, want = embedded_hash(so), source_hash(kind)
    if got != want:
        raise RuntimeError(f"{so.name} was built from other sources (embedded hash {got}, tree {want}); rebuild it "
                           "with `python -m transmogrifai_amd.ops.build --force`")


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
        if force or _stale(HOST_SO, "host"):
            tmp = HOST_SO.with_suffix(f".so.tmp{os.getpid()}")
            cxx = shutil.which("g++") or "c++"
            import sysconfig
            prov = _provenance_source("host", source_hash("host"))
            # utf8_pack.cpp reads str objects through the CPython API (symbols from the running interpreter)
            _run([cxx] + HOST_FLAGS + [f"-I{CSRC}", f"-I{sysconfig.get_paths()['include']}", "-o", str(tmp)] +
                 [str(s) for s in srcs] + [str(prov)])
            os.replace(tmp, HOST_SO)
            os.remove(prov)
    return HOST_SO


def build_hip(force: bool = False, arch: str = ARCH) -> Path:
    srcs = _sources("hip")
    hipcc = hipcc_path()
    if hipcc is None:
        raise RuntimeError("hipcc not found: cannot build the HIP kernels")
    with _Lock():
        if force or _stale(HIP_SO, "hip"):
            from concurrent.futures import ThreadPoolExecutor
            srcs = srcs + [_provenance_source("hip", source_hash("hip", arch))]
            objs = [str(LIB / (s.stem + ".o")) for s in srcs]
            # one hipcc per translation unit, a few at a time (the tree kernels alone take ~1 min)
            with ThreadPoolExecutor(max_workers=max(1, min(8, os.cpu_count() or 1))) as ex:
                list(ex.map(lambda so: _run([hipcc, f"--offload-arch={arch}"] + HIP_FLAGS +
                                            [f"-I{CSRC}", "-o", so[1], str(so[0])]),
                            zip(srcs, objs)))
            tmp = HIP_SO.with_suffix(f".so.tmp{os.getpid()}")
            _run([hipcc, f"--offload-arch={arch}", "-shared", "-fPIC", "-o", str(tmp)] + objs + ["-lrccl"])
            os.replace(tmp, HIP_SO)
            for o in objs + [str(srcs[-1])]:
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
