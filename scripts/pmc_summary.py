"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc_attn.sh) into per-kernel derived metrics.

usage: python scripts/pmc_summary.py gpurun_out/pmc > profiles/<name>.txt
"""
import collections
import csv
import glob
import os
import sys


def load(root):
    """Per program and kernel: counter sums, plus ``_ns_<counter>`` = summed dispatch time of the
    dispatches that carried that counter (for rates such as the effective clock)."""
    progs = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in sorted(glob.glob(os.path.join(root, "*_p*", "run_counter_collection.csv"))):
        prog = os.path.basename(os.path.dirname(f)).rsplit("_p", 1)[0]
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            k = k.replace("void ", "")[:48]
            c = r["Counter_Name"]
            progs[prog][k][c] += float(r["Counter_Value"])
            if "Start_Timestamp" in r:
                progs[prog][k]["_ns_" + c] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return progs


def ratio(a, b):
    return a / b if b else float("nan")


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    progs = load(root)
    hdr = ("kernel", "waves", "mfma_busy/busy", "valu/mfma", "lds_conf/lds", "wait_lds/wave_cyc",
           "active/wave_cyc", "wait_any/wave_cyc", "L2_hit", "clk_GHz")
    print("%-48s %8s %14s %10s %12s %17s %15s %17s %7s %8s" % hdr)
    for prog, kernels in progs.items():
        print(f"# {prog}")
        for k, c in kernels.items():
            if not c.get("SQ_INSTS_MFMA"):
                continue  # MFMA kernels only (skip RNG / fill kernels of the driver script)
            print("%-48s %8.0f %14.2f %10.1f %12.2f %17.3f %15.3f %17.3f %7.2f %8.3f" % (
                k, c["SQ_WAVES"],
                ratio(c["SQ_VALU_MFMA_BUSY_CYCLES"], c["SQ_BUSY_CYCLES"]),
                ratio(c["SQ_INSTS_VALU"], c["SQ_INSTS_MFMA"]),
                ratio(c["SQ_LDS_BANK_CONFLICT"], c["SQ_INSTS_LDS"]),
                ratio(c["SQ_WAIT_INST_LDS"], c["SQ_WAVE_CYCLES"]),
                ratio(c["SQ_ACTIVE_INST_ANY"], c["SQ_WAVE_CYCLES"]),
                ratio(c["SQ_WAIT_ANY"], c["SQ_WAVE_CYCLES"]),
                ratio(c["TCC_HIT_sum"], c["TCC_HIT_sum"] + c["TCC_MISS_sum"]),
                # effective clock: GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS)
                ratio(c["GRBM_GUI_ACTIVE"] / 8.0, c["_ns_GRBM_GUI_ACTIVE"])))


if __name__ == "__main__":
    main()
