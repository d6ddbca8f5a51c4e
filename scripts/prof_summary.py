"""Summarise a rocprofv3 kernel profile into a markdown table.

    # aggregate stats (every kernel of the run, divided by --steps)
    python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv --steps 2 --title "..."
    # one optimizer step cut out of the kernel trace: the kernels after the
    # second-to-last AdamW launch up to and including the last one (excludes
    # warmup, autotuner timing runs and eval)
    python scripts/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --last-step --title "..."
"""
import argparse
import collections
import csv

STEP_MARK = "adamw_kernel"


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("Cijk_") or n.startswith("Custom_Cijk"):
        return "hipBLASLt " + n.split("_UserArgs")[0][:60]
    return n.split("(")[0][:70]


def from_stats(path, steps):
    rows = list(csv.DictReader(open(path)))
    out = {}
    for r in rows:
        out[r["Name"]] = (float(r["TotalDurationNs"]) / steps, int(r["Calls"]) / steps)
    return out, None


def from_trace_last_step(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if STEP_MARK in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit(f"need >= 2 '{STEP_MARK}' launches in the trace, found {len(marks)}")
    # the step's AdamW may be several launches in a row: walk back over the run of marks
    last = marks[-1]
    j = len(marks) - 1
    while j > 0 and marks[j - 1] >= marks[j] - 4:
        j -= 1
    prev = marks[j - 1] if j > 0 else -1
    seg = rows[prev + 1:last + 1]
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in seg:
        a = agg[r["Kernel_Name"]]
        a[0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a[1] += 1
    wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
    return {k: (v[0], v[1]) for k, v in agg.items()}, wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=1, help="optimizer steps covered by a stats file")
    ap.add_argument("--last-step", action="store_true", help="input is a kernel trace; cut the last step")
    ap.add_argument("--title", default="kernel time")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    if a.last_step:
        data, wall = from_trace_last_step(a.csv)
    else:
        data, wall = from_stats(a.csv, a.steps)
    tot = sum(v[0] for v in data.values())
    print(f"## {a.title}\n")
    print(f"GPU kernel time {tot / 1e6:.1f} ms/step" + (f" (first-to-last kernel span {wall:.1f} ms)" if wall else "")
          + "\n")
    print("| kernel | ms/step | % | calls/step | avg us |")
    print("|---|---:|---:|---:|---:|")
    for name, (ns, calls) in sorted(data.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"| `{short(name)}` | {ns / 1e6:.2f} | {100 * ns / tot:.1f} | {calls:.0f} | {ns / max(calls, 1) / 1e3:.1f} |")


if __name__ == "__main__":
    main()
