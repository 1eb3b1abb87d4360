"""Copy the judged evidence of one tools/gpu.sh run from gpurun_out/ (scratch) into profiles/.

    python tools/save_run.py gpurun_out/r6h profiles/r6_h "gpurun -- bash tools/gpu.sh r6h ..." "(tree ...)"

Writes, under the profile directory:
  * COMMAND          the task list and the tree it ran (arguments 3 and 4)
  * SUMMARY.txt      tools/rank_brief.py's one line per run
  * <run>.json       the final JSON line of every bench / preset / service log
  * <run>/rank*.json the per-rank reports of ranks:N runs
  * suite.txt        the pytest verdict lines of suite runs
  * meminfo.log      the host page-cache / pressure samples (meminfo tasks)
  * roofline.md      tools/roofline.py over the run's pmc passes (when it has both roofline passes)
  * latency.md       tools/latency_breakdown.py over the run's first bench trace
  * profser_timeline.md  tools/gpu_timeline.py over the run's serialised kernel trace
"""
import glob
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def _last_json(path):
    for line in reversed(open(path, errors="replace").read().splitlines()):
        line = line.strip()
        if line.startswith("{") and line.endswith("}"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


def _tool(args, out):
    r = subprocess.run([sys.executable] + args, capture_output=True, text=True)
    if r.returncode == 0 and r.stdout.strip():
        with open(out, "w") as fh:
            fh.write(r.stdout)
        return True
    return False


def main(src, dst, command="", tree=""):
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, "COMMAND"), "w") as fh:
        fh.write(command.strip() + "\n" + (tree.strip() + "\n" if tree else ""))
    _tool([os.path.join(HERE, "rank_brief.py"), src], os.path.join(dst, "SUMMARY.txt"))
    for log in sorted(glob.glob(os.path.join(src, "*.log"))):
        name = os.path.basename(log)[:-4]
        if name.startswith("suite"):
            keep = [ln for ln in open(log, errors="replace").read().splitlines()
                    if " PASSED" in ln or " FAILED" in ln or " ERROR" in ln or "passed" in ln or "failed" in ln]
            with open(os.path.join(dst, "suite.txt" if name == "suite_2" else name + ".txt"), "w") as fh:
                fh.write("\n".join(keep) + "\n")
            continue
        if name.startswith(("pmc_", "profser_")):
            continue
        j = _last_json(log)
        if j is not None:
            with open(os.path.join(dst, name + ".json"), "w") as fh:
                json.dump(j, fh)
                fh.write("\n")
    for d in sorted(glob.glob(os.path.join(src, "ranks*"))):
        if os.path.isdir(d):
            for r in glob.glob(os.path.join(d, "rank*.json")):
                os.makedirs(os.path.join(dst, os.path.basename(d)), exist_ok=True)
                shutil.copy(r, os.path.join(dst, os.path.basename(d)))
    if os.path.exists(os.path.join(src, "meminfo.log")):
        shutil.copy(os.path.join(src, "meminfo.log"), dst)
    if len(glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True)) >= 2:
        _tool([os.path.join(HERE, "roofline.py"), src, "/dev/stdout", "24"], os.path.join(dst, "roofline.md"))
    traces = sorted(glob.glob(os.path.join(src, "trace_*.json")))
    if traces:
        _tool([os.path.join(HERE, "latency_breakdown.py"), traces[0]], os.path.join(dst, "latency.md"))
    ps = sorted(d for d in glob.glob(os.path.join(src, "profser_*")) if os.path.isdir(d))
    if ps:
        _tool([os.path.join(HERE, "gpu_timeline.py"), ps[0]], os.path.join(dst, "profser_timeline.md"))
    print("\n".join(sorted(os.listdir(dst))))


if __name__ == "__main__":
    main(*sys.argv[1:])
