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
        if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
            out.append(f"L2_hit={v['TCC_HIT_sum'] / max(1.0, v['TCC_HIT_sum'] + v['TCC_MISS_sum']):.0%}")
        if "FETCH_SIZE" in v:  # KB; gfx950 tallies 128-B streaming requests at 64 B (x2, MI355X_MICROARCH.md)
            out.append(f"fetch~{2 * v['FETCH_SIZE'] / 1e6:.2f}GB")
        out += [f"{c}={x:.3g}" for c, x in sorted(v.items())]
        print(" | ".join(out))


if __name__ == "__main__":
    main()
