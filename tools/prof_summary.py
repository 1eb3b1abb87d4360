"""rocprofv3 --stats kernel_stats.csv -> markdown table (short kernel names)."""
import csv
import re
import sys


def short(n):
    n = re.sub(r"rocprim::ROCPRIM_\w+::", "rocprim::", n).replace("(anonymous namespace)::", "")
    m = re.search(r"wrapped_(\w+?)_config", n)
    if "trampoline_kernel" in n and m:
        return "rocprim::" + m.group(1)
    return n.split("(")[0][:80]


def main(src, dst, title):
    rows = list(csv.DictReader(open(src)))
    with open(dst, "w") as f:
        f.write(f"# {title}\n\n")
        f.write("| kernel | calls | total us | avg us | % |\n|---|---|---|---|---|\n")
        for r in rows:
            f.write(f"| {short(r['Name'])} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e3:.1f} | "
                    f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "kernel stats")
