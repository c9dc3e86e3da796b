"""Per-launch HBM traffic of the MFMA kernels from a round_artifacts.sh output directory.

Reads the FETCH_SIZE (bench_p1) and WRITE_SIZE (bench_p2) rocprofv3 --pmc passes and writes
  profiles/<round>/pmc_bench_n2v_traffic.json   all kernels of interest
  (bench.py reads profiles/traffic_<workload>_<fn>.json: tools/roofline_evidence.py writes those)
bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts half of wide streaming
reads; MI355X_MICROARCH.md HBM section).
Usage: python tools/traffic_json.py gpurun_out/<tag> profiles/<round>"""
import collections
import csv
import json
import os
import sys

KERNELS = {  # key in the JSON -> (kernel-name substring, bench.py roofline name or None)
    "mlp_fused_fwd": ("mlp_fused_fwd", "mlp_fused_fwd"),
    "mlp_fused_dgrad": ("mlp_fused_fwd", None),  # same kernel symbol; split below by launch order
    "linear_wgrad_x3_wide": ("linear_wgrad_x3_wide", "linear_wgrad_x3"),
    "linear_wgrad_x3": ("linear_wgrad_x3_kernel", None),
}
METHOD = ("rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py --steps 5 "
          "--warmup 2 (tools/round_artifacts.sh); bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE "
          "counts half of wide streaming reads, MI355X_MICROARCH.md HBM section)")


def per_launch(d, counter):
    """{kernel-substring-key: [values in dispatch order]} for one pass directory."""
    rows = sorted(csv.DictReader(open(f"{d}/run_counter_collection.csv")), key=lambda r: int(r["Dispatch_Id"]))
    out = collections.defaultdict(list)
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        for key, (sub, _) in KERNELS.items():
            if key == "mlp_fused_dgrad":
                continue
            if sub in name:
                out[key].append(float(r["Counter_Value"]))
                break
    return out


def main(src, dst):
    fetch = per_launch(f"{src}/bench_p1", "FETCH_SIZE")
    write = per_launch(f"{src}/bench_p2", "WRITE_SIZE")
    res = {}
    for key in ["mlp_fused_fwd", "linear_wgrad_x3_wide", "linear_wgrad_x3"]:
        f, w = fetch.get(key, []), write.get(key, [])
        if not f or not w:
            continue
        if key == "mlp_fused_fwd":
            # one training step launches the fused kernel twice: the forward, then the
            # backward's input-gradient chain (n2v bench: no coarse pass)
            for k2, sl in (("mlp_fused_fwd", slice(0, None, 2)), ("mlp_fused_dgrad", slice(1, None, 2))):
                ff, ww = f[sl], w[sl]
                res[k2] = {"FETCH_SIZE_KB": sum(ff) / len(ff), "WRITE_SIZE_KB": sum(ww) / len(ww),
                           "launches": [len(ff), len(ww)]}
            continue
        res[key] = {"FETCH_SIZE_KB": sum(f) / len(f), "WRITE_SIZE_KB": sum(w) / len(w), "launches": [len(f), len(w)]}
    for v in res.values():
        v["bytes_per_launch"] = (2 * v["FETCH_SIZE_KB"] + v["WRITE_SIZE_KB"]) * 1024
    os.makedirs(dst, exist_ok=True)
    summary = os.path.join(dst, "pmc_bench_n2v_traffic.json")
    json.dump({"kernels": res, "method": METHOD, "source": src}, open(summary, "w"), indent=1)
    names = {"mlp_fused_fwd": ("mlp_fused_fwd", "mlp_fused_fwd (the forward launches of the default bench command)"),
             "mlp_fused_dgrad": ("mlp_fused_dgrad",
                                 "mlp_fused_dgrad (the input-gradient-chain launches of the default bench command)"),
             "linear_wgrad_x3_wide": ("linear_wgrad_x3",
                                      "linear_wgrad_x3 (weight-gradient GEMMs, wide launches of the default bench command)")}
    for key, (fname, desc) in names.items():
        if key in res:
            out = dict(kernel=desc, **res[key], method=METHOD, source=summary)
            json.dump(out, open(os.path.join("profiles", f"traffic_{fname}.json"), "w"), indent=1)
    for k, v in res.items():
        print(f"{k}: {v['bytes_per_launch'] / 1e6:.1f} MB/launch ({v['launches']})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
