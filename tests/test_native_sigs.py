"""Every native entry point the Python side calls has a declared ctypes signature (ops/_native.py): an undeclared
one passes 64-bit pointers as C ints and faults on the device box, not here."""
import pathlib
import re

from transmogrifai_amd.ops import _native as N

_INLINE = {"tmog_hip_set_oom_handler", "tmog_utf8_copy", "tmog_utf8_offsets"}   # argtypes set where loaded


def test_every_called_native_function_is_declared():
    root = pathlib.Path(N.__file__).resolve().parents[1]
    known = set(N._HOST_SIGS) | set(N._HIP_SIGS) | _INLINE
    missing = {}
    for p in root.rglob("*.py"):
        for m in re.finditer(r"\.(tmog_\w+)\s*\(", p.read_text()):
            if m.group(1) not in known and not m.group(1).endswith("_source_hash"):
                missing.setdefault(m.group(1), set()).add(p.name)
    assert not missing, missing


def test_declared_arity_matches_the_hip_sources():
    src = "\n".join(p.read_text() for p in (pathlib.Path(N.__file__).parent / "csrc" / "hip").glob("*.hip"))
    for name, args in N._HIP_SIGS.items():
        m = re.search(r"\b(?:int|void|size_t|int64_t|void\*)\s+" + name + r"\s*\(([^)]*)\)\s*\{", src)
        if m is None:
            continue
        params = [a for a in m.group(1).split(",") if a.strip()]
        assert len(params) == len(args), (name, len(params), len(args))
