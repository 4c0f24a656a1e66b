"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (mean over dispatches):
busy ratios (MFMA busy per CU-cycle, VALU / LDS issue), LDS bank-conflict share, instruction mix per MFMA.

    python scripts/pmc_summary.py gpurun_out/pmc_attn/p1/p1_counter_collection.csv gpurun_out/pmc_attn/p2/... \
        --match flash_ --cus 256
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="", help="regex on the kernel name")
    ap.add_argument("--cus", type=int, default=256)
    # GRBM_GUI_ACTIVE comes back summed over the XCDs (8 on MI355X): divide for the kernel's cycle count
    ap.add_argument("--xcds", type=int, default=8)
    args = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in args.csv:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if args.match and not re.search(args.match, name):
                continue
            per[(name, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for (name, _), cs in per.items():
            for c, v in cs.items():
                vals[re.sub(r"^void ", "", name)[:90]][c].append(v)
    for name, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"## {name}")
        for c in sorted(m):
            print(f"  {c:28s} {m[c]:.4g}")
        g = m.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            cyc = g / args.xcds
            print(f"  -> MFMA busy {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * args.cus * 4):.1%} of SIMD-cycles "
                  f"({cyc:.4g} cycles per pass)")
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            print(f"  -> LDS bank-conflict cycles {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.1%} of LDS-array cycles")
        if m.get("SQ_INSTS_MFMA"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
                if c in m:
                    print(f"  -> {c[9:]} per MFMA {m[c] / m['SQ_INSTS_MFMA']:.2f}")
        if m.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    print(f"  -> {c[3:]} / wave-cycles {m[c] / m['SQ_WAVE_CYCLES']:.1%}")


if __name__ == "__main__":
    main()
