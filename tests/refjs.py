"""Helpers to run the reference's own JavaScript through tests/js/ref_harness.js."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
HARNESS = os.path.join(HERE, "js", "ref_harness.js")


def run(req: dict):
    env = dict(os.environ, TZ="UTC")
    r = subprocess.run(["node", HARNESS], input=json.dumps(req), capture_output=True, text=True,
                       env=env, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-4000:])
    return json.loads(r.stdout)


def parse(batch_list):
    req = {"mode": "parse",
           "batches": [{"now": now, "chunks": [[fp, ls] for fp, ls in chunks]} for now, chunks in batch_list]}
    return run(req)


def stats(lines):
    return run({"mode": "stats", "lines": lines})


def zscore(config_text, lines, reloads=()):
    """reloads: [(line index, config text)] applied as the reference's watcher does."""
    return run({"mode": "zscore", "configText": config_text, "lines": lines,
                "reloads": [{"at": a, "configText": t} for a, t in reloads]})


def alerts(config_text, lines, clock="entry", reloads=()):
    return run({"mode": "alerts", "configText": config_text, "lines": lines, "clock": clock,
                "reloads": [{"at": a, "configText": t} for a, t in reloads]})


def util(**kw):
    return run(dict(mode="util", **kw))
