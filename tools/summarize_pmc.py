"""Summarize a `tools/gpu/run.sh gemmpmc` run: per GEMM shape (qkv, out, ffn1, ffn2 — tools/gemm_pmc.py's
order, dispatched round robin) the kernel-trace median, and from the PMC passes:
  wave-cycle split (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES, all in
  quad-cycles): parked on s_waitcnt / barrier, issue-stalled, issuing;
  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); held clock;
  instructions per wave, LDS bank-conflict cycles / LDS-array cycles;
  HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE KiB (gfx950 FETCH_SIZE reports half of wide reads).

    python tools/summarize_pmc.py gpurun_out/<tag> [shapes]
"""
import collections
import csv
import glob
import json
import os
import sys

ALG = {"qkv": (65536, 2304, 768), "out": (65536, 768, 768), "ffn1": (65536, 3072, 768), "ffn2": (65536, 768, 3072),
       "ffn1b": (65536, 3072, 768)}


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        out += list(csv.DictReader(open(f)))
    out.sort(key=lambda r: int(r["Dispatch_Id"]))
    return out


def main():
    d = sys.argv[1]
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(ALG)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    tr = [r for r in rows(os.path.join(d, "trace", "**", "*kernel_trace.csv")) if "k_gemm" in r["Kernel_Name"]]
    for i, r in enumerate(tr):
        per[names[i % len(names)]]["dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for p in sorted(glob.glob(os.path.join(d, "pmc*"))):
        if not os.path.isdir(p):
            continue
        seen = []
        for r in rows(os.path.join(p, "**", "*counter_collection.csv")):
            if "k_gemm" not in r["Kernel_Name"]:
                continue
            if r["Dispatch_Id"] not in seen:
                seen.append(r["Dispatch_Id"])
            t = names[(len(seen) - 1) % len(names)]
            per[t][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                per[t]["pmc_dur"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {}
    for t in names:
        v = per[t]
        mean = {k: sum(x) / len(x) for k, x in v.items() if x}
        dur = sorted(v["dur_ns"])
        med = dur[len(dur) // 2] / 1e3 if dur else None
        M, N, K = ALG[t]
        r = {"median_us": med, "tflops": round(2 * M * N * K / (med * 1e-6) / 1e12, 1) if med else None}
        if med:
            r["frac_2p5"] = round(r["tflops"] / 2500, 4)
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if k in mean:
                    r[k.lower().replace("sq_", "") + "_frac"] = round(mean[k] / wc, 4)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and "GRBM_GUI_ACTIVE" in mean:
            r["mfma_busy"] = round(mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (mean["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
            if v["pmc_dur"]:
                r["clock_ghz"] = round(mean["GRBM_GUI_ACTIVE"] / 8 / (sum(v["pmc_dur"]) / len(v["pmc_dur"])), 3)
        waves = mean.get("SQ_WAVES")
        if waves:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SALU"):
                if k in mean:
                    r[k.lower().replace("sq_insts_", "per_wave_")] = round(mean[k] / waves, 1)
        if "SQ_LDS_BANK_CONFLICT" in mean and mean.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_conflict_frac"] = round(mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_LDS_IDX_ACTIVE"], 4)
        if "FETCH_SIZE" in mean:
            r["read_MB"] = round(2 * 1024 * mean["FETCH_SIZE"] / 1e6, 1)
            r["read_x_alg"] = round(r["read_MB"] * 1e6 / (2 * (M * K + N * K)), 2)
        if "WRITE_SIZE" in mean:
            r["write_MB"] = round(1024 * mean["WRITE_SIZE"] / 1e6, 1)
        for k, x in mean.items():
            if k not in ("dur_ns", "pmc_dur") and not k.startswith("SQ_") and k not in ("FETCH_SIZE", "WRITE_SIZE",
                                                                                     "GRBM_GUI_ACTIVE"):
                r[k] = x
        res[t] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
