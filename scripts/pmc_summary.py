"""Per-kernel averages of a rocprofv3 --pmc CSV (counter collection), as one table row
per kernel: raw counters plus derived fractions (wave-cycle shares, MFMA busy per SIMD).

    python scripts/pmc_summary.py gpurun_out/pmc/p1_counter_collection.csv [p2...] --match flash
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in a.csv:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            if a.match and a.match not in name:
                continue
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in agg.items():
        v = {c: sum(x) / len(x) for c, x in cs.items()}
        out = [name]
        wc = v.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in v:
                    out.append(f"{c[3:]}={v[c] / wc:.0%}")
        if "GRBM_GUI_ACTIVE" in v and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
            cyc = v["GRBM_GUI_ACTIVE"] / 8
            out.append(f"mfma_busy/SIMD={v['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc:.0%}")
        out += [f"{c}={x:.3g}" for c, x in sorted(v.items())]
        print(" | ".join(out))


if __name__ == "__main__":
    main()
