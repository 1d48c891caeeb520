"""Hash of the library sources (mass-raytrace_amd/csrc + include): the Makefile
bakes it into libmassrt.so (mrt_build_info), bench.py / smoke() compare the
loaded library's value with the tree's, and PMC summaries are stamped with it.

  python tools/src_hash.py      # prints the 16-hex-digit hash
"""
from __future__ import annotations

import hashlib
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
SRC_DIRS = [REPO / "mass-raytrace_amd" / "csrc", REPO / "include"]


def src_hash() -> str:
    h = hashlib.sha256()
    for d in SRC_DIRS:
        for p in sorted(d.rglob("*")):
            if p.is_file() and p.suffix in (".h", ".hip", ".cpp"):
                h.update(str(p.relative_to(REPO)).encode())
                h.update(p.read_bytes())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(src_hash())
