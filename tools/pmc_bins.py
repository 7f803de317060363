#!/usr/bin/env python3
"""Dev tool: per-bin counter table of the task kernels.

    python tools/pmc_bins.py OUTDIR KS_LOG CALIB_JSON DST_JSON

OUTDIR/pmc*/ hold rocprofv3 --pmc passes over ONE phased scale-22 product (tools/phase_timing.py
SCALE 1) and over the merge sample (tools/merge_sample.py); KS_LOG is a plain phase_timing run whose
last line is the library's per-kind stats {kind: {ms, launches, alg_bytes}} of one product.
Per bin (kernel configuration): launches, kernel ms, algorithmic GB/s, FETCH/WRITE bytes (raw and
with the calibrated FETCH factor), HBM GB/s, L2 hit rate, LDS bank-conflict fraction
(SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE), wait fraction and SALU/VALU.
"""
import ast
import collections
import csv
import glob
import json
import re
import sys

PAT = re.compile(r"task_kernel<cbh::(\w+)<(\w+)>, (\d+), (\d+), (\d+), (\d+), (\d+)(?:, (true|false))?>")
MODES = {0: "sym", 1: "num", 2: "dense"}


def bin_of(name):
    if "merge2_kernel<" in name:  # device/merge2.h (round 6): two-list merge path, count / write pass
        return "merge_num" if ", true," in name else "merge_sym"
    if "dense_kernel<" in name:  # device/dense_kernel.h (round 5): numeric dense / symbolic bitmap
        m = re.search(r"dense_kernel<.*, (\d+)>", name.split("(")[0])
        kind = m.group(1) if m else "?"
        return {"0": "num_dense", "1": "sym_bmp", "2": "num_large"}.get(kind, "dense_" + kind)
    m = PAT.search(name)
    if not m:
        return None
    T, BS, EMAX, U, mode = (int(m.group(i)) for i in range(3, 8))
    merge = m.group(8) == "true"
    kind = MODES[mode]
    if merge:
        return "merge_" + kind
    if kind == "dense":
        return "num_dense"
    return f"{kind}_{'large' if BS == 512 else 'small'}"


def main(src, ks_log, calib_json, dst):
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    names = {}
    for f in sorted(glob.glob(src + "/pmc*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            b = bin_of(r["Kernel_Name"])
            if b is None:
                continue
            names[b] = r["Kernel_Name"].split("(")[0].replace("void ", "")
            sums[b][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(b, r["Counter_Name"])].add(r["Dispatch_Id"])
    ks = {}
    for line in open(ks_log):
        if line.startswith("{"):
            ks = ast.literal_eval(line.strip())
    calib = json.load(open(calib_json))["kernels"] if calib_json != "-" else {}
    rows = {}
    for b, c in sorted(sums.items()):
        k = ks.get(b, {})
        ms = k.get("ms", 0.0)
        n = len(disp.get((b, "FETCH_SIZE"), ())) or k.get("launches", 0)
        fetch = c.get("FETCH_SIZE", 0.0) * 1024
        write = c.get("WRITE_SIZE", 0.0) * 1024
        row = {
            "kernel": names[b], "dispatches_profiled": n,
            "kernel_ms": round(ms, 3) if ms else None, "launches_timed": k.get("launches"),
            "alg_bytes": k.get("alg_bytes"),
            "alg_GBps": round(k["alg_bytes"] / ms / 1e6, 1) if ms and k.get("alg_bytes") else None,
            "fetch_bytes_raw": round(fetch), "write_bytes": round(write),
            "hbm_bytes_raw": round(fetch + write), "hbm_bytes_x2": round(2 * fetch + write),
            "hbm_GBps_raw": round((fetch + write) / ms / 1e6, 1) if ms else None,
            "hbm_GBps_x2": round((2 * fetch + write) / ms / 1e6, 1) if ms else None,
            "traffic_over_alg_raw": round((fetch + write) / k["alg_bytes"], 3) if k.get("alg_bytes") else None,
            "traffic_over_alg_x2": round((2 * fetch + write) / k["alg_bytes"], 3) if k.get("alg_bytes") else None,
        }
        if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum"):
            row["l2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_bank_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
        if c.get("SQ_WAVE_CYCLES"):
            row["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 4)
        if c.get("SQ_INSTS_VALU"):
            row["salu_over_valu"] = round(c.get("SQ_INSTS_SALU", 0) / c["SQ_INSTS_VALU"], 4)
        row["counters_sum"] = {a: v for a, v in sorted(c.items())}
        rows[b] = row
    out = {"bins": rows, "calibration": calib, "source": src, "ks_log": ks_log}
    json.dump(out, open(dst, "w"), indent=1)
    hdr = f"{'bin':10s} {'ms':>8s} {'algGB/s':>8s} {'hbmGB/s raw/x2':>16s} {'traf/alg raw/x2':>16s} {'L2hit':>6s} {'LDSconf':>7s} {'wait':>6s} {'S/V':>6s}"
    print(hdr)
    for b, r in rows.items():
        f = lambda x: "-" if x is None else x  # noqa: E731
        print(f"{b:10s} {f(r['kernel_ms'])!s:>8s} {f(r['alg_GBps'])!s:>8s} "
              f"{f(r['hbm_GBps_raw'])!s:>7s}/{f(r['hbm_GBps_x2'])!s:<8s} "
              f"{f(r['traffic_over_alg_raw'])!s:>7s}/{f(r['traffic_over_alg_x2'])!s:<8s} "
              f"{f(r.get('l2_hit_rate'))!s:>6s} {f(r.get('lds_bank_conflict_frac'))!s:>7s} "
              f"{f(r.get('wait_frac'))!s:>6s} {f(r.get('salu_over_valu'))!s:>6s}")


if __name__ == "__main__":
    main(*sys.argv[1:])
