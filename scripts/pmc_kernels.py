#!/usr/bin/env python3
"""Summarise scripts/profile_round.sh's rocprofv3 runs into profiles/pmc_kernels.json (read by
bench.py's roofline) and profiles/<tag>_<config>_{kernel_stats.csv,kernels.json}.

Per config and kernel (names as bench.py / cwbl_kernel_times give them):
  avg_ms                 rocprofv3 --kernel-trace --stats average duration
  hbm_bytes_per_launch   (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 from separate --pmc passes;
                         on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
                         reads (MI355X_MICROARCH.md, HBM section), so 2 x FETCH_SIZE is the
                         corrected read volume (an upper estimate for mixed-width reads)
  fp64_flops_per_launch  64 x (2 FMA_F64 + ADD_F64 + MUL_F64 + TRANS_F64) + 512 x MFMA_MOPS_F64
  points_per_launch      from the profiled bench run's own kernel timing (detail.kernels_rank0)
  fp64_flops_per_point   the ratio of the two
"""
import csv
import glob
import json
import os
import shutil
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").replace("cwbl::", "").strip()


def counters(path):
    agg = {}
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def bench_line(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def main(src, tag):
    path = os.path.join("profiles", "pmc_kernels.json")
    pm = json.load(open(path)) if os.path.exists(path) else {}
    pm["tag"] = tag
    pm["formula"] = __doc__.split("Per config")[1].strip()
    pm.setdefault("configs", {})
    for cdir in sorted(glob.glob(os.path.join(src, "*"))):
        cfg = os.path.basename(cdir)
        stats = {}
        ks = os.path.join(cdir, "kt", "kt_kernel_stats.csv")
        if not os.path.exists(ks):
            continue
        for r in csv.DictReader(open(ks)):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]),
                                       "avg_ms": float(r["AverageNs"]) / 1e6}
        fetch = counters(os.path.join(cdir, "fetch", "fetch_counter_collection.csv"))
        write = counters(os.path.join(cdir, "write", "write_counter_collection.csv"))
        f64 = counters(os.path.join(cdir, "f64", "f64_counter_collection.csv"))
        b = bench_line(os.path.join(cdir, "f64.log")) or {}
        kern = (b.get("detail") or {}).get("kernels_rank0", {})
        out = {}
        for k, st in stats.items():
            e = dict(st)
            if k in fetch:
                e["hbm_bytes_per_launch"] = (2 * fetch[k]["FETCH_SIZE"] +
                                             write.get(k, {}).get("WRITE_SIZE", 0.0)) * 1024
            if k in f64:
                m = f64[k]
                e["counters_per_launch"] = m
                e["fp64_flops_per_launch"] = 64 * (
                    2 * m.get("SQ_INSTS_VALU_FMA_F64", 0) + m.get("SQ_INSTS_VALU_ADD_F64", 0) +
                    m.get("SQ_INSTS_VALU_MUL_F64", 0) + m.get("SQ_INSTS_VALU_TRANS_F64", 0)) + \
                    512 * m.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0)
            if k in kern and kern[k]["launches"]:
                e["points_per_launch"] = kern[k]["points"] / kern[k]["launches"]
                if "fp64_flops_per_launch" in e and e["points_per_launch"]:
                    e["fp64_flops_per_point"] = e["fp64_flops_per_launch"] / e["points_per_launch"]
            out[k] = e
        out["_meta"] = {"steps": 1}  # profile_round.sh profiles one step (--steps 1 --warmup 0)
        pm["configs"][cfg] = out
        os.makedirs("profiles", exist_ok=True)
        shutil.copy(ks, f"profiles/{tag}_{cfg}_kernel_stats.csv")
        json.dump({"tag": tag, "config": cfg, "bench": b, "kernels": out},
                  open(f"profiles/{tag}_{cfg}_kernels.json", "w"), indent=1)
        print(cfg, json.dumps({k: {a: v for a, v in e.items() if a != "counters_per_launch"}
                               for k, e in out.items() if "fp64_flops_per_launch" in e}, indent=1))
    json.dump(pm, open(path, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
