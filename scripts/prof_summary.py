"""Summarise a rocprofv3 --stats kernel_stats.csv into a markdown table.

    python scripts/prof_summary.py gpurun_out/prof2/run_kernel_stats.csv --steps 2 --title "..." > profiles/x.md
"""
import argparse
import csv


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("Cijk_") or n.startswith("Custom_Cijk"):
        return "hipBLASLt " + n.split("_UserArgs")[0][:60]
    return n.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=1, help="optimizer steps covered by the trace")
    ap.add_argument("--title", default="kernel time")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"## {a.title}\n")
    print(f"Total GPU kernel time {tot / 1e6:.1f} ms over {a.steps} step(s) = {tot / 1e6 / a.steps:.1f} ms/step\n")
    print("| kernel | ms/step | % | calls/step | avg us |")
    print("|---|---:|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: a.top]:
        print(f"| `{short(r['Name'])}` | {float(r['TotalDurationNs']) / 1e6 / a.steps:.2f} | "
              f"{float(r['Percentage']):.1f} | {int(r['Calls']) / a.steps:.0f} | {float(r['AverageNs']) / 1e3:.1f} |")


if __name__ == "__main__":
    main()
