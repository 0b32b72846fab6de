"""Summarise a tools/gpu_profile.sh run into profiles/<tag>_summary.md + CSVs.

Per kernel: calls, average duration (kernel trace), HBM bytes per launch from
FETCH_SIZE/WRITE_SIZE (KB units; FETCH doubled per the gfx950 correction in
MI355X_MICROARCH.md §HBM), achieved GB/s, and fp32 MFMA FLOPs per launch from
SQ_INSTS_VALU_MFMA_MOPS_F32 (x512, counter_defs MfmaFlopsF32).
    python tools/pmc_summary.py gpurun_out/prof_r1 profiles/r1
"""
import csv
import shutil
import sys
from collections import defaultdict
from pathlib import Path


def short(name):
    n = name.replace("void ", "")
    return n.split("(")[0]


def load_counter(path, counters):
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] in counters:
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r["Dispatch_Id"])
    return agg, {k: len(v) for k, v in calls.items()}


def main(src, dst):
    src, dst = Path(src), Path(dst)
    dst.parent.mkdir(parents=True, exist_ok=True)
    stats = list(csv.DictReader(open(src / "trace" / "run_kernel_stats.csv")))
    shutil.copy(src / "trace" / "run_kernel_stats.csv", f"{dst}_kernel_stats.csv")
    fetch, nf = load_counter(src / "pmc_FETCH_SIZE" / "run_counter_collection.csv", {"FETCH_SIZE"})
    write, nw = load_counter(src / "pmc_WRITE_SIZE" / "run_counter_collection.csv", {"WRITE_SIZE"})
    mf, nm = load_counter(src / "pmc_SQ_INSTS_VALU_MFMA_MOPS_F32" / "run_counter_collection.csv",
                          {"SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"})
    rows = []
    total_ns = sum(float(s["TotalDurationNs"]) for s in stats)
    for s in stats:
        k = short(s["Name"])
        avg_ns = float(s["AverageNs"])
        fb = 2 * 1024 * fetch[k]["FETCH_SIZE"] / max(nf.get(k, 1), 1)
        wb = 1024 * write[k]["WRITE_SIZE"] / max(nw.get(k, 1), 1)
        flop = 512 * mf[k]["SQ_INSTS_VALU_MFMA_MOPS_F32"] / max(nm.get(k, 1), 1)
        busy = mf[k]["SQ_VALU_MFMA_BUSY_CYCLES"]
        gui = mf[k]["GRBM_GUI_ACTIVE"]
        rows.append(dict(kernel=k, calls=int(s["Calls"]), pct=float(s["Percentage"]),
                         avg_us=avg_ns / 1e3, hbm_mb=(fb + wb) / 1e6,
                         gbps=(fb + wb) / avg_ns, tflops=flop / avg_ns / 1e3,
                         mfma_util=(busy / (gui * 4 * 256 / 8) if gui else 0.0)))
    with open(f"{dst}_summary.md", "w") as f:
        f.write(f"# rocprofv3 summary ({src.name})\n\n")
        f.write("Per-launch averages. HBM = 2*FETCH_SIZE + WRITE_SIZE (gfx950 read correction); "
                "TFLOP/s from SQ_INSTS_VALU_MFMA_MOPS_F32*512; profiled passes run at reduced "
                "clocks (DVFS), so trace durations are the reference for time.\n\n")
        f.write("| kernel | calls | % time | avg µs | HBM MB/launch | GB/s | MFMA TFLOP/s |\n|---|---|---|---|---|---|---|\n")
        for r in sorted(rows, key=lambda r: -r["pct"]):
            f.write(f"| {r['kernel'][:70]} | {r['calls']} | {r['pct']:.1f} | {r['avg_us']:.1f} | "
                    f"{r['hbm_mb']:.2f} | {r['gbps']:.0f} | {r['tflops']:.1f} |\n")
        f.write(f"\nTotal kernel time {total_ns / 1e6:.1f} ms over the profiled run.\n")
    print(open(f"{dst}_summary.md").read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
