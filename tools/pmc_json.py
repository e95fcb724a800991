#!/usr/bin/env python3
"""PMC passes of one bench workload -> profiles/pmc_c3.json (read by bench.py's roofline).

Input: the directory written by tools/gpu_pmc.sh: pass directories p*/ (rocprofv3 --pmc
counter_collection.csv of `bench.py --steps 1 --warmup 0 --capture 0 --no-cpu-baseline`), the
bench's own JSON line in p*.log (its config, so bench.py can check that the counters belong to
the config it runs), and calib/ (tools/valu_calib under the SQ pass).

Per kernel, averaged over its dispatches:
  hbm_bytes_per_dispatch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
      (MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports 1/2 of the bytes of 16-B-per-lane
      reads — the traversal's node/triangle/ray loads are dwordx4; WRITE_SIZE is exact for 16-B
      stores; the unit is kB)
  valu_issue_frac = 2 * SQ_INSTS_VALU / (SIMDS * GRBM_GUI_ACTIVE / XCDS)
      the fraction of the SIMDs' VALU issue cycles the kernel's wave64 VALU instructions take,
      at 2 cycles each (CDNA4 SIMDs are 32 lanes wide: MI355X_MICROARCH.md, `v_fma_f32` wave64
      2 cyc); SQ_INSTS_VALU counts wave-level VALU instructions summed over the GPU (the
      calibration kernel's count equals its instruction count exactly); GRBM_GUI_ACTIVE is the
      GPU-busy cycle count summed over the 8 XCDs (/8 -> cycles of the dispatch); SIMDS = 256
      CUs x 4. Packed (v_pk_*) instructions take 4 cycles and transcendentals 8, so for mixed
      code this is a lower bound of the issue-cycle share.
  valu_busy = 4 * SQ_ACTIVE_INST_VALU / (SIMDS * GRBM_GUI_ACTIVE / XCDS)   (rounds 2-6 headline)
      SQ_ACTIVE_INST_VALU counts quad-cycles (x4 -> cycles). The calibration kernel
      (tools/valu_calib.hip) compiles to v_pk_fma_f32 — 4 cycles per wave64 instruction — and
      reads 0.83; for unpacked code the quad-cycle count is 2x the issue cycles, so this figure
      overstates issue utilization up to 2x and can exceed 1 (the round-6 closest-hit kernel
      reads 1.03). Kept for comparison with earlier rounds' records.
  l2_hit = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

SIMDS, XCDS = 256 * 4, 8
# k_occluded (batch E) and k_order_* (batch H's shading-order variant): rejected experiments,
# kept here so that their committed PMC records can be regenerated from the variant builds
KERNELS = {"k_trace<false>": "k_trace<false", "k_trace<true>": "k_trace<true", "k_occluded": "k_occluded",
           "k_shade": "k_shade<", "k_raygen": "k_raygen", "k_order_count": "k_order_count",
           "k_order_scatter": "k_order_scatter", "k_shadow_resolve": "k_shadow_resolve",
           "k_resolve_pixels": "k_resolve_pixels", "k_fill_paths": "k_fill_paths", "k_valu_calib": "k_valu_calib"}


def per_dispatch(dirs):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for d in dirs:
        for f in Path(d).rglob("*counter_collection.csv"):
            for row in csv.DictReader(open(f)):
                name = row.get("Kernel_Name", "")
                # the fused depth-0 instantiations (k_trace<false, false, 1..4>) apart
                prim = re.search(r"k_trace<false, \w+, [1-4]>", name) is not None
                for k, tag in KERNELS.items():
                    if k == "k_trace<false>" and prim:
                        k = "k_trace<false> depth 0 fused"
                    if tag in name:
                        c = row["Counter_Name"]
                        acc[k][c] += float(row["Counter_Value"] or 0)
                        disp[k][c].add((str(f), row.get("Dispatch_Id", "")))
    out = {}
    for k in acc:
        out[k] = {c: acc[k][c] / max(1, len(disp[k][c])) for c in acc[k]}
        out[k]["dispatches"] = max(len(v) for v in disp[k].values())
    return out


def derive(c):
    d = dict(c)
    if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
        d["hbm_bytes_per_dispatch"] = 2.0 * 1024.0 * c.get("FETCH_SIZE", 0.0) + 1024.0 * c.get("WRITE_SIZE", 0.0)
    if c.get("GRBM_GUI_ACTIVE") and "SQ_ACTIVE_INST_VALU" in c:
        d["valu_busy"] = 4.0 * c["SQ_ACTIVE_INST_VALU"] / (SIMDS * c["GRBM_GUI_ACTIVE"] / XCDS)
    if c.get("GRBM_GUI_ACTIVE") and "SQ_INSTS_VALU" in c:
        d["valu_issue_frac"] = 2.0 * c["SQ_INSTS_VALU"] / (SIMDS * c["GRBM_GUI_ACTIVE"] / XCDS)
    if "TCC_HIT_sum" in c and (c["TCC_HIT_sum"] + c.get("TCC_MISS_sum", 0)) > 0:
        d["l2_hit"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if c.get("SQ_THREAD_CYCLES_VALU") and c.get("SQ_ACTIVE_INST_VALU"):
        # thread-cycles per VALU instruction cycle; / the calibration kernel's (64 active lanes)
        d["thread_cycles_per_valu_cycle"] = c["SQ_THREAD_CYCLES_VALU"] / c["SQ_ACTIVE_INST_VALU"]
    if c.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c:
                d[k.lower() + "_frac_of_wave_cycles"] = c[k] / c["SQ_WAVE_CYCLES"]
    return d


def main(root, out):
    root = Path(root)
    passes = sorted(p for p in root.glob("p*") if p.is_dir())
    config = None
    for log in sorted(root.glob("p*.log")):
        for line in open(log):
            if line.startswith("{") and '"metric"' in line:
                config = json.loads(line)["config"]
    kern = {k: derive(v) for k, v in per_dispatch(passes).items() if k != "k_valu_calib"}
    calib = per_dispatch([root / "calib"]).get("k_valu_calib") if (root / "calib").exists() else None
    full = derive(calib).get("thread_cycles_per_valu_cycle") if calib else None
    if full:
        # VALU lane utilization: active lanes per issued VALU cycle, relative to a kernel whose
        # every lane is active; useful_valu_frac = valu_issue_frac x lane utilization
        for k, v in kern.items():
            if "thread_cycles_per_valu_cycle" in v:
                v["valu_lane_util"] = v["thread_cycles_per_valu_cycle"] / full
                if "valu_issue_frac" in v:
                    v["useful_valu_frac"] = v["valu_issue_frac"] * v["valu_lane_util"]
    res = {"source": "rocprofv3 --pmc, one pass per counter group (tools/gpu_pmc.sh), bench.py --steps 1 "
                     "--warmup 0 --capture 0 --no-cpu-baseline",
           "formulas": {"hbm_bytes_per_dispatch": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024",
                        "valu_issue_frac": f"2*SQ_INSTS_VALU / ({SIMDS} SIMDs * GRBM_GUI_ACTIVE/{XCDS}): 2 issue "
                                           "cycles per wave64 VALU instruction on a 32-wide SIMD (lower bound: "
                                           "packed ops take 4, transcendentals 8)",
                        "valu_busy": f"4*SQ_ACTIVE_INST_VALU / ({SIMDS} SIMDs * GRBM_GUI_ACTIVE/{XCDS}) (quad-cycle "
                                     "count; 2x the issue cycles of unpacked code, rounds 2-6 records)",
                        "l2_hit": "TCC_HIT_sum/(TCC_HIT_sum+TCC_MISS_sum)",
                        "valu_lane_util": "(SQ_THREAD_CYCLES_VALU/SQ_ACTIVE_INST_VALU) / the same ratio of the "
                                          "calibration kernel (all 64 lanes active)",
                        "useful_valu_frac": "valu_issue_frac * valu_lane_util"},
           "config": config, "kernels": kern,
           "calibration": derive(calib) if calib else None}
    Path(out).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
