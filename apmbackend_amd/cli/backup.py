"""Source backup (reference ``backup.sh``: copy ``*.js`` to ``js_bkups/<name>.<YYYYMMDDHH>``).

Copies the package's Python and C++/HIP sources plus the config into
``<dest>/<relative path>.<YYYYMMDDHH>``.

Usage: python -m apmbackend_amd.cli.backup [--dest DIR]
"""
from __future__ import annotations

import argparse
import datetime as _dt
import glob
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PATTERNS = ["apmbackend_amd/**/*.py", "apmbackend_amd/csrc/**/*.h", "apmbackend_amd/csrc/**/*.cpp",
            "apmbackend_amd/csrc/**/*.hip", "config/*.json", "bench.py", "__graft_entry__.py"]


def backup(dest: str, root: str = ROOT, stamp: str = None) -> list:
    stamp = stamp or _dt.datetime.now().strftime("%Y%m%d%H")
    done = []
    for pat in PATTERNS:
        for src in glob.glob(os.path.join(root, pat), recursive=True):
            rel = os.path.relpath(src, root)
            dst = os.path.join(dest, f"{rel}.{stamp}")
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copy2(src, dst)
            done.append(dst)
    return sorted(done)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="backup")
    ap.add_argument("--dest", default=os.path.join(ROOT, "src_bkups"))
    a = ap.parse_args(argv)
    n = len(backup(a.dest))
    print(f"{n} files backed up to {a.dest}")
    return 0


if __name__ == "__main__":  # pragma: no cover
    sys.exit(main())
