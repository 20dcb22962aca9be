"""Per-op rocprofv3 counters of the replay kernels -> profiles/pmc_counters_config<N>.json.

Input: the counter_collection CSVs of separate `rocprofv3 --pmc ...` passes over the same
`bench.py --config N --steps 1 --warmup 0 --no-cpu` command (scripts/gpu_check.sh pmcA/pmcB/pmcf/
pmcw<N>), and that command's bench log (its JSON line gives the ops each replay launch applied).
Counters are summed over the instances (XCD / SE) of a dispatch and over the dispatches of the
kernel in the profiled step (one step, no warmup: config 3 launches each class twice, one launch
per half), and divided by the ops all of those launches applied.

Derived per kernel:
  per_op[c]         counter / ops applied by the launch
  ipc_per_wave      instructions / (SQ_WAVE_CYCLES * 4): SQ cycle counters count quad-cycles
                    (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC units")
  lds_bytes_per_op  SQ_LDS_IDX_ACTIVE (LDS-array cycles, all CUs) x 256 B / ops: the bytes the LDS
                    array could have moved in the cycles it was busy for this kernel (256 B per
                    array cycle, MI355X_MICROARCH.md §LDS) -- the LDS roofline's numerator
  hbm_bytes         (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)

usage: python tools/pmc_counters.py --config N --bench-log LOG --out OUT CSV [CSV ...]
"""
import argparse
import collections
import csv
import json
import re


def read_counters(paths):
    acc = collections.defaultdict(float)  # (kernel, dispatch, counter) -> value summed over instances
    for p in paths:
        for r in csv.DictReader(open(p)):
            key = (r["Kernel_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")), r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
    per = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> [per dispatch]
    for (k, _, c), v in acc.items():
        per[k][c].append(v)
    # every dispatch of the profiled step (config 3: the two halves' launches of a class) summed,
    # pairing with the ops all of the class's launches applied (bench line)
    return {k: {c: sum(v) for c, v in cs.items()} for k, cs in per.items()}


def bench_line(path):
    for ln in open(path):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            return json.loads(ln)
    raise SystemExit(f"no bench JSON line in {path}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--bench-log", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("csv", nargs="+")
    a = ap.parse_args()
    line = bench_line(a.bench_log)
    ops_by_class = collections.defaultdict(int)
    for li in line["launches"]:
        ops_by_class[li["seg_class"]] += li["ops"]
    cnt = read_counters(a.csv)
    opd = line["config"]["ops_per_doc"]  # config 4: {"min", "max", "lpt_loads"} (bench.py's n_ops is the max)
    res = {"config": a.config, "docs": line["config"]["docs_per_gpu"], "ops": opd["max"] if isinstance(opd, dict) else opd,
           "command": "bench.py --config %d --docs %d --steps 1 --warmup 0 --no-cpu" % (a.config, line["config"]["docs_per_gpu"]),
           "units": "counters summed over instances and over the step's dispatches of the kernel; per_op = / ops its launches applied",
           "kernels": {}}
    for k, cs in sorted(cnt.items()):
        m = re.match(r"mt_replay_kernel_(\d+)", k)
        if not m or int(m.group(1)) not in ops_by_class:
            continue
        ops = ops_by_class[int(m.group(1))]
        ent = {"ops": ops, "counters": cs, "per_op": {c: round(v / ops, 3) for c, v in cs.items()}}
        insts = sum(cs.get(c, 0.0) for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM",
                                            "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"))
        if insts and cs.get("SQ_WAVE_CYCLES"):
            ent["insts_per_op"] = round(insts / ops, 1)
            ent["ipc_per_wave"] = round(insts / (4.0 * cs["SQ_WAVE_CYCLES"]), 4)
        if cs.get("SQ_LDS_IDX_ACTIVE"):
            ent["lds_bytes_per_op"] = round(cs["SQ_LDS_IDX_ACTIVE"] * 256.0 / ops, 1)
        if "FETCH_SIZE" in cs or "WRITE_SIZE" in cs:
            ent["hbm_bytes"] = (2 * cs.get("FETCH_SIZE", 0.0) + cs.get("WRITE_SIZE", 0.0)) * 1024
            ent["hbm_bytes_per_op"] = round(ent["hbm_bytes"] / ops, 1)
        res["kernels"][k] = ent
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: {x: v.get(x) for x in ("insts_per_op", "ipc_per_wave", "lds_bytes_per_op", "hbm_bytes_per_op")}
                      for k, v in res["kernels"].items()}))


if __name__ == "__main__":
    main()
