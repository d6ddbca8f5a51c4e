"""Per-dispatch breakdown of the last optimizer step of a rocprofv3 kernel trace.

Cuts the kernels between the last two AdamW launches, groups dispatches by
(kernel, grid, workgroup) and prints time per group — grid sizes separate the
GEMM shapes that share one kernel name, so each training GEMM gets its own row.

    python scripts/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--top 60]
"""
import argparse
import collections
import csv

STEP_MARK = "adamw_kernel"


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("Cijk_") or n.startswith("Custom_Cijk"):
        return "hipBLASLt " + n.split("_UserArgs")[0][:48]
    return n.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if STEP_MARK in r["Kernel_Name"]]
    seg = rows[marks[-2] + 1:marks[-1] + 1]
    wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
    agg = collections.defaultdict(lambda: [0.0, 0, None])
    busy = 0.0
    for r in seg:
        g = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        key = (short(r["Kernel_Name"]), g, int(r["Workgroup_Size_X"]))
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        agg[key][0] += d
        agg[key][1] += 1
        agg[key][2] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"])
        busy += d
    print(f"step span {wall:.2f} ms, kernel busy {busy:.2f} ms, {len(seg)} dispatches")
    print(f"| kernel | grid (wg) | wg | calls | ms | avg us | vgpr/agpr/lds |")
    print("|---|---|---:|---:|---:|---:|---|")
    for (name, g, wg), (ms, n, res) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"| `{name}` | {g[0]}x{g[1]}x{g[2]} | {wg} | {n} | {ms:.2f} | {ms / n * 1000:.1f} | {'/'.join(res)} |")


if __name__ == "__main__":
    main()
