"""Process memory probe (reference ``pid_stats.py``: ps_mem 3.13 with ``-m`` and ``-q``).

The supervisor's ``pidInspectionCommand`` runs ``pid_stats -p <PID> -S -q -m`` and parses the
quiet line ``"<ram> MiB <swap> MiB"`` (apm_manager.js:359-370).  RAM is the proportional set
size (PSS) and swap the SwapPss, read from ``/proc/<pid>/smaps_rollup`` (or summed over
``smaps``) -- the native reader in csrc/runtime/procstat.cpp when the extension is built.
New: ``-g`` adds the HBM the process holds (KFD sysfs), the MI355X-side memory of an engine.

Usage: python -m apmbackend_amd.cli.pid_stats -p PID[,PID...] [-S] [-q] [-m] [-t] [-g]
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import Optional, Tuple


def _read_kb(path: str, keys=("Pss:", "SwapPss:")) -> Optional[Tuple[int, int]]:
    pss = swap = 0
    found = False
    try:
        with open(path) as f:
            for line in f:
                if line.startswith(keys[0]):
                    pss += int(line.split()[1])
                    found = True
                elif line.startswith(keys[1]):
                    swap += int(line.split()[1])
    except OSError:
        return None
    return (pss, swap) if found else None


def pss_swap_bytes(pid) -> Tuple[Optional[int], Optional[int]]:
    for name in ("smaps_rollup", "smaps"):
        r = _read_kb(f"/proc/{pid}/{name}")
        if r is not None:
            return r[0] * 1024, r[1] * 1024
    return None, None


def human(num_bytes: float, units: Optional[float]) -> str:
    """ps_mem human(): MiB with one decimal in -m mode, else an auto-scaled unit."""
    if units:
        return "%.1f" % (num_bytes / units)
    power = 1024.0
    for unit in ("KiB", "MiB", "GiB", "TiB"):
        num_bytes /= power
        if num_bytes < power:
            return "%.1f %s" % (num_bytes, unit)
    return "%.1f PiB" % (num_bytes / power)


def vram_bytes(pid) -> int:
    from ..runtime.supervisor import pid_vram_mb
    return int(pid_vram_mb(int(pid)) * 2**20)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="pid_stats", description=__doc__.splitlines()[0])
    ap.add_argument("-p", dest="pids", required=True, help="comma-separated PIDs")
    ap.add_argument("-S", "--swap", action="store_true", help="show swap usage")
    ap.add_argument("-q", "--quiet", action="store_true", help="only '<ram> <unit> <swap> <unit>' per pid")
    ap.add_argument("-m", "--mb", action="store_true", help="MiB units")
    ap.add_argument("-t", "--total", action="store_true", help="only the total")
    ap.add_argument("-g", "--gpu", action="store_true", help="also report HBM held by the process (new)")
    a = ap.parse_args(argv)
    units = 1024.0 * 1024.0 if a.mb else None
    unit = "MiB" if a.mb else ""
    total = total_swap = 0
    rows = []
    for p in a.pids.split(","):
        p = p.strip()
        if not p:
            continue
        try:
            from .. import _native
            pss, swap = _native.load(build_if_missing=False).pid_pss_swap(int(p))
            if pss < 0:
                pss = swap = None
        except Exception:
            pss, swap = pss_swap_bytes(p)
        if pss is None:
            sys.stderr.write(f"pid {p} not found or not readable\n")
            return 1
        total += pss
        total_swap += swap
        rows.append((p, pss, swap))
    if a.total:
        sys.stdout.write(f"{human(total, units)} {unit} {human(total_swap, units)} {unit}\n".replace("  ", " "))
        return 0
    for p, pss, swap in rows:
        if a.quiet:
            line = f"{human(pss, units)} {unit} {human(swap, units)} {unit}"
        else:
            line = f"{human(pss, units):>9} {unit}"
            if a.swap:
                line += f"   {human(swap, units):>9} {unit}"
            line += f"\tpid[{p}]"
        if a.gpu:
            line += f" {human(vram_bytes(p), units)} {unit}"
        sys.stdout.write(line.rstrip() + "\n")
    return 0


if __name__ == "__main__":  # pragma: no cover
    sys.exit(main())
