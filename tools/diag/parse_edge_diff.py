"""Diagnostic (GPU): K1/K2 events of the edge corpus vs the Python model, both parse kernels;
prints the lines whose events differ (by chunk, line) with their text."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from test_engine_gpu import KINDS, START, UTC, _edge_corpus, small_cfg  # noqa: E402

from apmbackend_amd.models.oracle import file_kind  # noqa: E402
from apmbackend_amd.models.pipeline import APMEngine  # noqa: E402
from apmbackend_amd.ops.parse_ref import EVENT_DTYPE, parse_batch  # noqa: E402

for seed in (3, 4):
    for mode in (("line", "tile") if os.environ.get("DIAG_TILE") else ("line",)):
        os.environ["APM_PARSE"] = mode
        files = _edge_corpus(seed)
        eng = APMEngine(small_cfg(), keep_text=False)
        raw = [(fp, ("\n".join(ls) + "\n").encode("utf-8")) for fp, ls in files.items()]
        eng.process(raw, START + 60_000)
        got = np.frombuffer(eng.eng.last_events(), dtype=EVENT_DTYPE)
        bch = [(KINDS[file_kind(fp)], b) for fp, b in raw]
        cf = [eng.file_ids[fp] for fp, _ in raw]
        want, _, _, _ = parse_batch(bch, UTC, {}, cf)
        g = {(int(e["chunk"]), int(e["line"])): e for e in got}
        w = {(int(e["chunk"]), int(e["line"])): e for e in want}
        extra = sorted(set(g) - set(w))
        miss = sorted(set(w) - set(g))
        bad = []
        for k in sorted(set(g) & set(w)):
            for name in EVENT_DTYPE.names:
                a, b = g[k][name], w[k][name]
                if not (a == b or (isinstance(a, float) and a != a and b != b)):
                    bad.append((k, name, a, b))
        print(f"seed {seed} mode {mode}: got {len(got)} want {len(want)} extra {len(extra)} missing {len(miss)} fielddiff {len(bad)}")
        allines = {}
        for ci, (fp, b) in enumerate(raw):
            allines[ci] = b.decode("utf-8").split("\n")
        # line index is the batch-global line number: map via cumulative counts
        cum, base = {}, 0
        for ci in range(len(raw)):
            cum[ci] = base
            base += len(allines[ci]) - 1
        def text(k):
            ci, li = k
            for cj in range(len(raw)):
                if cum[cj] <= li < cum[cj] + len(allines[cj]) - 1:
                    return repr(allines[cj][li - cum[cj]][:160])
            return "?"
        for k in extra[:8]:
            print("  EXTRA", k, "kind", g[k]["kind"], "mask", hex(g[k]["mask"]), text(k))
        for k in miss[:8]:
            print("  MISS ", k, "kind", w[k]["kind"], "mask", hex(w[k]["mask"]), text(k))
        for k, name, a, b in bad[:12]:
            print("  DIFF ", k, name, a, b, text(k))
