"""Summarize a tools/profile_bench.sh run into per-kernel-tag numbers.

Kernel trace -> average duration per tag; FETCH_SIZE / WRITE_SIZE passes -> HBM bytes per
dispatch. MI355X_MICROARCH.md (HBM / rocprofv3): both counters are in KiB, and on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads, so reads are doubled:
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.

GEMM dispatches are tagged like bench.py's HIP-event tags (gemm_qkv, gemm_out, gemm_ffn1,
gemm_ffn2, ...) from the epilogue template argument and the dispatch order within a layer.
Usage: python tools/summarize_profile.py gpurun_out/prof_r01 [--json out.json] [--config B,L,layers]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

EPI_TAG = {1: "gemm_qkv", 2: "gemm_ffn1", 3: "gemm_out", 4: "gemm_cos"}
RENAME = {"k_add_ln_split": "layernorm"}  # split-stream residual LayerNorm = bench tag "layernorm"
SIMPLE = ("k_band_attn", "k_gfold_partial", "k_gfold_qu", "k_gfold_u", "k_gfold_out", "k_layernorm",
          "k_embed_ln", "k_prepare", "k_gather_rows", "k_row_inv_norm", "k_cos_cand",
          "k_global_attn", "k_gemm_f32", "k_gemm_skinny", "k_band_attn_wide")


def tagger():
    last = [None]

    def tag(name, grid):
        m = re.search(r"k_gemm_bf16<(\d+), (\d+), \d+, \d+, \d+, \d+, (\d+),", name)
        # 256^2 persistent kernels (ping-pong / four-wave): mangled (..Li<epi>E..) or demangled with
        # the epilogue as the first integer argument; rocprofv3 garbles some demangled names of the
        # 16-bit-templated kernels ("<bool _Accum, int, E, ...>"), which are bias epilogues here
        mm = re.search(r"k_gemm_(?:pp|w4r?)I(?:DF16b|DF16_|f)Li(\d+)E", name)
        md = re.search(r"k_gemm_(?:pp|w4r?)<(\d+)?", name)
        mp = mm or md
        if m or mp:
            if m:
                bm, epi = int(m.group(1)), int(m.group(3))
            else:
                bm, epi = 256, int(mp.group(1)) if mp.group(1) else 1
            if epi == 5:  # residual + LN recompute epilogue (training / older runs)
                t = "gemm_ffn2" if last[0] == "gemm_ffn1" else "gemm_out"
            elif epi == 1 and bm == 128:
                t = "gemm_qg"
            elif epi == 1:  # bias epilogue: qkv, out-proj and FFN2 by their order in a layer
                t = {"gemm_ffn1": "gemm_ffn2", "gemm_qkv": "gemm_out"}.get(last[0], "gemm_qkv")
            else:
                t = EPI_TAG.get(epi, f"gemm_epi{epi}")
            last[0] = t
            return t
        for k, t in RENAME.items():
            if k in name:
                return t
        for k in SIMPLE:
            if k in name:
                return k[2:]
        return "other:" + name[:40]
    return tag


def load_dispatches(pattern):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def main():
    out = sys.argv[1]
    jpath = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else os.path.join(out, "summary.json")
    per = collections.defaultdict(lambda: {"calls": 0, "dur_ns": 0.0, "durs": [], "FETCH_SIZE": [], "WRITE_SIZE": [],
                                           "SQ_VALU_MFMA_BUSY_CYCLES": [], "GRBM_GUI_ACTIVE": [],
                                           "SQ_BUSY_CYCLES": []})
    tag = tagger()
    for r in load_dispatches(os.path.join(out, "trace", "**", "*kernel_trace.csv")):
        t = tag(r["Kernel_Name"], int(r.get("Grid_Size", 0) or 0))
        per[t]["calls"] += 1
        per[t]["dur_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per[t]["durs"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for kind in ("fetch", "write", "mfma"):
        tag = tagger()
        last_id, t = None, None
        for r in load_dispatches(os.path.join(out, kind, "**", "*counter_collection.csv")):
            if r["Dispatch_Id"] != last_id:  # a pass with several counters has one row per counter
                last_id = r["Dispatch_Id"]
                t = tag(r["Kernel_Name"], int(r["Grid_Size"]))
            per[t][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                per[t].setdefault("pmc_durs", []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(v["dur_ns"] for v in per.values())
    res = {}
    for t, v in per.items():
        if not v["calls"]:
            continue
        f, w = v["FETCH_SIZE"], v["WRITE_SIZE"]
        rb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        # MFMA busy: SQ_VALU_MFMA_BUSY_CYCLES (per-SIMD busy cycles, summed over the chip) over the
        # SIMD-cycles of the dispatch: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 x 256 CUs x 4 SIMDs
        mb, ga = v["SQ_VALU_MFMA_BUSY_CYCLES"], v["GRBM_GUI_ACTIVE"]
        # the PMC pass's own per-dispatch durations give the clock (GRBM_GUI_ACTIVE / 8 per second)
        pd = v.setdefault("pmc_durs", [])
        busy = None
        if mb and ga and len(mb) == len(ga):
            busy = round(sum(mb) / (sum(ga) / 8 * 256 * 4), 4)
        d = sorted(v["durs"])
        res[t] = {"calls": v["calls"], "avg_us": round(v["dur_ns"] / v["calls"] / 1e3, 2),
                  "median_us": round(d[len(d) // 2] / 1e3, 2), "mfma_busy": busy,
                  "clock_ghz": round(sum(ga) / 8 / sum(pd), 3) if ga and pd and len(pd) == len(ga) else None,
                  "share": round(v["dur_ns"] / total, 4),
                  "hbm_read_bytes": rb, "hbm_write_bytes": wb,
                  "hbm_bytes": (rb + wb) if rb is not None and wb is not None else None}
    print(f"{'tag':24s} {'calls':>6s} {'avg_us':>9s} {'med_us':>9s} {'share':>6s} {'HBM MB/launch':>14s} "
          f"{'GB/s':>7s} {'MFMA busy':>9s}")
    for t, r in sorted(res.items(), key=lambda kv: -kv[1]["share"]):
        hb = r["hbm_bytes"]
        mb = r["mfma_busy"]
        print(f"{t:24s} {r['calls']:6d} {r['avg_us']:9.1f} {r['median_us']:9.1f} {100 * r['share']:6.2f} "
              f"{hb / 1e6 if hb else float('nan'):14.1f} {hb / r['median_us'] / 1e3 if hb else float('nan'):7.0f} "
              f"{mb if mb is not None else float('nan'):9.3f}")
    cfg = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "64,1024,12"
    B, L, layers = (int(x) for x in cfg.split(","))
    json.dump({"config": {"batch": B, "seq_len": L, "layers": layers},
               "source": "rocprofv3 --kernel-trace --stats, then --pmc FETCH_SIZE, --pmc WRITE_SIZE and --pmc "
                         "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES in separate passes; "
                         "hbm = (2*FETCH_SIZE + WRITE_SIZE) KiB; mfma_busy = MFMA_BUSY / (GRBM_GUI_ACTIVE/8 * 1024)",
               "tags": res}, open(jpath, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
