"""Summarise a tools/gpu_profile.sh run into profiles/<tag>_summary.md + CSVs.

Per kernel: calls, average duration (kernel trace), HBM bytes per launch from
FETCH_SIZE/WRITE_SIZE (KB units; FETCH doubled per the gfx950 correction in
MI355X_MICROARCH.md §HBM), achieved GB/s, and fp32 MFMA FLOPs per launch from
SQ_INSTS_VALU_MFMA_MOPS_F32 (x512, counter_defs MfmaFlopsF32).
    python tools/pmc_summary.py gpurun_out/prof_r1 profiles/r1
"""
import csv
import json
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
    if not Path(path).exists():  # pass not collected in this run
        return agg, {}
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
                          {"SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_INSTS_VALU_MFMA_MOPS_BF16",
                           "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"})
    stall_f = src / "pmc_SQ_WAVE_CYCLES" / "run_counter_collection.csv"
    stall_c = {"SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
               "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS"}
    stall, _ = load_counter(stall_f, stall_c) if stall_f.exists() else ({}, {})
    rows = []
    total_ns = sum(float(s["TotalDurationNs"]) for s in stats)
    for s in stats:
        k = short(s["Name"])
        avg_ns = float(s["AverageNs"])
        fb = 2 * 1024 * fetch[k]["FETCH_SIZE"] / max(nf.get(k, 1), 1)
        wb = 1024 * write[k]["WRITE_SIZE"] / max(nw.get(k, 1), 1)
        flop = 512 * mf[k]["SQ_INSTS_VALU_MFMA_MOPS_F32"] / max(nm.get(k, 1), 1)
        flop_bf16 = 512 * mf[k].get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) / max(nm.get(k, 1), 1)
        busy = mf[k]["SQ_VALU_MFMA_BUSY_CYCLES"]
        gui = mf[k]["GRBM_GUI_ACTIVE"]
        rows.append(dict(kernel=k, calls=int(s["Calls"]), pct=float(s["Percentage"]),
                         avg_us=avg_ns / 1e3, hbm_mb=(fb + wb) / 1e6,
                         hbm_bytes=fb + wb, gbps=(fb + wb) / avg_ns, tflops=flop / avg_ns / 1e3,
                         tflops_bf16=flop_bf16 / avg_ns / 1e3,
                         mfma_util=(busy / (gui * 4 * 256 / 8) if gui else 0.0)))
    with open(f"{dst}_summary.md", "w") as f:
        f.write(f"# rocprofv3 summary ({src.name})\n\n")
        f.write("Per-launch averages. HBM = 2*FETCH_SIZE + WRITE_SIZE (gfx950 read correction); "
                "hardware MFMA TFLOP/s from SQ_INSTS_VALU_MFMA_MOPS_{F32,BF16}*512 (the split-bf16 "
                "kernels issue 6 bf16 products per fp32-accurate MAC, so their bf16 rate is 6x the "
                "algorithmic rate); profiled passes run at reduced clocks (DVFS), so trace durations "
                "are the reference for time.\n\n")
        f.write("| kernel | calls | % time | avg µs | HBM MB/launch | GB/s | MFMA f32 TF/s | MFMA bf16 TF/s |\n|---|---|---|---|---|---|---|---|\n")
        for r in sorted(rows, key=lambda r: -r["pct"]):
            if nf:
                f.write(f"| {r['kernel'][:70]} | {r['calls']} | {r['pct']:.1f} | {r['avg_us']:.1f} | "
                        f"{r['hbm_mb']:.2f} | {r['gbps']:.0f} | {r['tflops']:.1f} | {r['tflops_bf16']:.1f} |\n")
            else:  # kernel trace + stall pass only
                f.write(f"| {r['kernel'][:70]} | {r['calls']} | {r['pct']:.1f} | {r['avg_us']:.1f} | "
                        f"n/a | n/a | n/a | n/a |\n")
        f.write(f"\nTotal kernel time {total_ns / 1e6:.1f} ms over the profiled run.\n")
        if stall:
            f.write("\nWave-cycle split (SQ_WAIT_ANY = parked at s_waitcnt/barrier, SQ_WAIT_INST_ANY = "
                    "issue stall incl. waiting for the busy MFMA pipe, SQ_ACTIVE_INST_ANY = issuing) and "
                    "LDS bank-conflict cycles per LDS instruction, kernels > 1 % of time:\n\n"
                    "| kernel | wait_any | wait_inst | active | bank-conflict cyc / LDS inst |\n|---|---|---|---|---|\n")
            for r in sorted(rows, key=lambda r: -r["pct"]):
                c = stall.get(r["kernel"])
                if not c or r["pct"] < 1.0 or not c.get("SQ_WAVE_CYCLES"):
                    continue
                wc = c["SQ_WAVE_CYCLES"]
                f.write(f"| {r['kernel'][:70]} | {c.get('SQ_WAIT_ANY', 0) / wc:.2f} | "
                        f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} | {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} | "
                        f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_INSTS_LDS', 0), 1):.2f} |\n")
    if not nf:  # no traffic passes: keep the newest committed PMC JSON as the traffic source
        print(open(f"{dst}_summary.md").read())
        return
    json.dump({r["kernel"]: {"calls": r["calls"], "avg_us": round(r["avg_us"], 3),
                             "hbm_bytes": round(r["hbm_bytes"]), "gbps": round(r["gbps"], 1),
                             "mfma_f32_tflops": round(r["tflops"], 2),
                             "mfma_bf16_tflops": round(r["tflops_bf16"], 2)} for r in rows},
              open(f"{dst}_pmc.json", "w"), indent=1)
    print(open(f"{dst}_summary.md").read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
