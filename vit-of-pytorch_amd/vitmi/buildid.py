"""Source fingerprint of libvit_hip.so.

The Makefile stamps `tree_id()` of the sources it compiles into the library (`vit_build_id()`, csrc/capi.hip);
`vitmi._lib.load()` recomputes it from the tree next to the package and refuses a library built from
other sources, so a stale prebuilt .so (same ABI number, older kernels) cannot pass silently.

    python3 vitmi/buildid.py [package root]     # prints the id (the Makefile's call)
"""
from __future__ import annotations

import hashlib
import os
import sys

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


SOURCE_SUFFIXES = (".hip", ".h", ".inc")  # what the Makefile compiles or includes from csrc/


def source_files(pkg_root: str = PKG_ROOT) -> list[str]:
    """Every file the library is built from, relative to the package root, in a fixed order: the
    Makefile, each HIP source / header / include of csrc/ (not editor swap or backup files that may
    sit beside them), the C-ABI header."""
    csrc = os.path.join(pkg_root, "csrc")
    files = ["Makefile"] + [os.path.join("csrc", f) for f in sorted(os.listdir(csrc))
                            if f.endswith(SOURCE_SUFFIXES) and not f.startswith(".")
                            and os.path.isfile(os.path.join(csrc, f))]
    return files + [os.path.join("..", "include", "vit_hip.h")]


def tree_id(pkg_root: str = PKG_ROOT) -> str:
    """16 hex digits of SHA-256 over (relative path, contents) of source_files()."""
    h = hashlib.sha256()
    for rel in source_files(pkg_root):
        h.update(rel.replace(os.sep, "/").encode())
        h.update(b"\0")
        with open(os.path.join(pkg_root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def have_sources(pkg_root: str = PKG_ROOT) -> bool:
    return os.path.isdir(os.path.join(pkg_root, "csrc")) and os.path.isfile(os.path.join(pkg_root, "Makefile"))


if __name__ == "__main__":
    print(tree_id(sys.argv[1] if len(sys.argv) > 1 else PKG_ROOT))
