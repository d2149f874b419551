"""The product build's identity: a hash of the sources librtamd.so and the
pybind module are built from (csrc/, the Makefile, include/rt_render.h).

bench.py reports it and takes the roofline's PMC traffic only from a
profiles/ summary whose `build` field carries the same id (tools/profile.sh
writes it), so the counters always describe the benched kernels. No git:
the GPU box receives the tree without .git.
"""
import hashlib
import os

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_REPO = os.path.dirname(_PKG)


def source_files():
    files = [os.path.join(_PKG, "Makefile"), os.path.join(_REPO, "include", "rt_render.h")]
    for root, dirs, names in os.walk(os.path.join(_PKG, "csrc")):
        dirs.sort()
        files += [os.path.join(root, n) for n in sorted(names) if not n.endswith((".o", ".so", ".pyc"))]
    return files


def build_id():
    """12 hex digits of the sha256 over the source files' paths and bytes."""
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, _REPO).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]


if __name__ == "__main__":
    print(build_id())
