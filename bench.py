"""Headline benchmark: BP-decoded shots/s on hgp_34_n1600 (BASELINE.json `metric`).

One *step* = one fused Monte Carlo launch (``qldpc_mc_launch``) over a batch of
``--shots`` shots per GPU of the reference's code-capacity shot loop
(``CodeSimulator_DataError._single_run``, src/Simulators.py:117-168, as driven
by ``CodeFamily.EvalWER('data')``, :759-777): depolarizing Pauli error with
probabilities ``[p/3]*3`` where ``p = eval_p*3/2``, syndromes on hz and hx, two
min-sum BP decodes (alpha=0.625, max_iter=int(N/10)=160 -- the notebooks'
settings), residual and logical check, ``eval_logical_type='Total'``.  The
counters stay on the device and are all-reduced over RCCL once at the end (the
only collective of the path).

Run as ``python bench.py`` (N=1) or under ``torch.distributed.run`` with one
rank per GPU; shots are sharded by global shot index (weak scaling: every rank
decodes ``--shots`` shots per step).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Headline operating point: BP-only crossing region of the synthetic (3,4) HGP
# family under this decoder (tools/threshold_scan.py).
DEFAULT_P = 0.06
SEED = 0x51D5EED0 + 2  # seed = 0x51D5EED0 + config_id (config 2)

# Peaks.  HBM 8 TB/s (spec).  LDS-bound kernels: the ceiling of the kernel family's OWN per-row LDS
# instruction mix from the guide's cycle table (MI355X_MICROARCH.md §LDS: ds_read_b64 2, ds_read_b128 4,
# ds_write_b64 6, ds_write_b128 13 cycles per wave-instruction, one LDS array per CU, 256 CUs at
# 2.4 GHz), in algorithmic bytes: 64 lanes x edges x 32 B (fp64) per wave-row / the row's cycles.  The
# continuous-issue microbenchmark (tools/calib/lds_peak.hip, profiles/r05/calib/lds_peak.jsonl)
# reproduces the table's pure-read rates (ds_read_b64 147, ds_read_b128 155 TB/s at 16 waves per CU;
# guide ~150) and measures the m2s / m2s8 mixes at 89.1 / 91.4 TB/s (12 waves per CU): reported as
# `peak_measured`; `peak` is the (higher) guide-table ceiling.  LDS_PEAK_GBS (the guide's aggregate for
# 4-byte traffic) stays as `peak_guide_aggregate` for comparison with rounds 1-4.
LDS_PEAK_GBS = 75_000.0
HBM_PEAK_GBS = 8_000.0
LDS_CALIB = os.path.join(ROOT, "profiles", "r05", "calib", "lds_peak.jsonl")
_LDS_CYC = {"ds_read_b64": 2, "ds_read_b128": 4, "ds_write_b32": 4, "ds_write_b64": 6, "ds_write_b128": 13}
# per family: (edges per row, {instruction: count per wave-row}, calib mode or None, description
# [, algorithmic bytes per edge-iteration: 32 in fp64 (default), 16 in fp32])
LDS_MIX = {
    "f32w": (7, {"ds_read_b64": 7, "ds_read_b128": 2, "ds_write_b32": 7, "ds_write_b64": 1}, None,
             "fp32 two-word row of 7 in 2 chunks (engine id 3, compile-time 2-chunk rows, own v2c in VGPRs: the "
             "headline code's fp32 fast mode): 7 x (CS gather b64 + v2c store b32) + the row (2 x b128) + the CS "
             "store (b64) = 56 cycles per 7 x 16 B x 64 lanes", 16),
    "m2s": (7, {"ds_read_b64": 15, "ds_read_b128": 3, "ds_write_b64": 9}, "m2s_row_mix",
            "m2s row of 7 (engine id 11103): 7 x (CS gather b64 + V-slot read b64 + v2c store b64) + the row "
            "(3 x b128 + tail b64) + CS / argmin-slot stores (2 x b64) = 96 cycles"),
    "m2s8": (8, {"ds_read_b64": 16, "ds_read_b128": 4, "ds_write_b64": 10}, "m2s8_row_mix",
             "m2s8 row of 8 (engine ids 10103 / 10203): 8 x (b64 + b64 + store b64) + 4 x b128 + 2 x store b64 = 108 cycles"),
    "st64m2s": (9, {"ds_read_b64": 19, "ds_read_b128": 4, "ds_write_b64": 11}, None,
                "fp64 one-word tail row of 9 (engine ids 11313 / 111313, round 6: 1024-thread workgroups, own v2c "
                "in VGPRs): 9 x (CS gather b64 + V-slot read b64 + v2c store b64) + the row (4 x b128 + tail b64) + "
                "CS / argmin-slot stores (2 x b64) = 120 cycles"),
    "st64": (9, {"ds_read_b64": 10, "ds_read_b128": 13, "ds_write_b64": 9, "ds_write_b128": 1}, None,
             "fp64 two-word tail row of 9 (engine ids 1013 / 101013; 1024-thread workgroups, 128-VGPR budget: the "
             "own previous v2c is re-read from LDS, bp_reg.h RState::kKeepV false): 9 x (CS gather b128 + own V-slot "
             "read b64 + v2c store b64) + the row (4 x b128 + tail b64) + the CS store (b128) = 139 cycles"),
}


def lds_ceiling(kind):
    """(GB/s algorithmic, provenance dict) of an LDS-bound kernel family's row mix."""
    edges, mix, mode, what = LDS_MIX[kind][:4]
    bpe = LDS_MIX[kind][4] if len(LDS_MIX[kind]) > 4 else 32
    cyc = sum(_LDS_CYC[k] * v for k, v in mix.items())
    gbs = 64 * edges * bpe / cyc * 256 * 2.4  # B per cycle per CU x CUs x GHz
    prov = {"family": kind, "mix": mix, "cycles_per_wave_row": cyc, "algorithmic_bytes_per_wave_row": 64 * edges * bpe,
            "what": what, "source": "MI355X_MICROARCH.md §LDS cycle table, 256 CUs x 2.4 GHz"}
    if mode:
        try:
            best = None
            for line in open(LDS_CALIB):
                d = json.loads(line)
                if d.get("mode") == mode and d.get("workgroups_per_cu") == 3:
                    best = d
            if best:
                prov["measured"] = {"algorithmic_GBs": best["algorithmic_TBps"] * 1e3, "file": os.path.relpath(LDS_CALIB, ROOT),
                                    "how": "tools/calib/lds_peak.hip, continuous issue, 12 waves per CU"}
        except (OSError, ValueError, KeyError):
            pass
    return gbs, prov


def mix_of_kernel(kernel_id, precision, row_width=None):
    """The LDS_MIX family of an engine-3 kernel id (None: no row-mix ceiling derived; the guide aggregate)."""
    if precision == 32 and kernel_id == 3 and row_width == 7:
        return "f32w"
    if precision != 64 or kernel_id is None:
        return None
    if kernel_id == 11103:
        return "m2s"
    if kernel_id in (10103, 10203):
        return "m2s8"
    if kernel_id % 100000 in (1013, 101013) or kernel_id in (1013, 101013):
        return "st64"
    if kernel_id % 100000 == 11313:
        return "st64m2s"
    return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--code", default="hgp_34_n1600")
    ap.add_argument("--p", type=float, default=DEFAULT_P)
    ap.add_argument("--shots", type=int, default=1 << 18, help="shots per GPU per step")
    ap.add_argument("--precision", type=int, default=64, choices=(32, 64),
                    help="64 = ldpc's float64 arithmetic (the reference; headline), 32 = fast mode (not the reference)")
    ap.add_argument("--fp32-line", type=int, default=1,
                    help="also time the fp32 fast mode on the same workload (reported beside the headline, N=1)")
    ap.add_argument("--pmc-traffic", type=int, default=1,
                    help="measure HBM bytes per launch with rocprofv3 PMC passes of this build (N=1, before GPU init)")
    ap.add_argument("--max-iter-ratio", type=float, default=10)
    ap.add_argument("--logical", default="Total", choices=("X", "Z", "Total"))
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--comm", default="torch", choices=("torch", "native"),
                    help="torch: one rank per GPU (torchrun), counters all-reduced by torch.distributed; native: ONE "
                         "process drives --gpus GPUs through the C ABI (qldpc_mc_run_sharded + qldpc_comm_init_all)")
    ap.add_argument("--workload", default="data", choices=("data", "phenl", "bposd", "circuit"),
                    help="data = headline (config 2); phenl = space-time phenomenological (config 5)")
    ap.add_argument("--num-rep", type=int, default=3)
    ap.add_argument("--dem-d", type=int, default=3,
                    help="circuit workload: toric distance (3 = the demo's hgp(ring_code(3), ring_code(3)))")
    ap.add_argument("--circuit-noise", default="cx", choices=("cx", "all"),
                    help="circuit workload: CX noise only (the demo) or every noise source at p")
    ap.add_argument("--sampler", default="skip", choices=("skip", "keyed"),
                    help="circuit workload: DEM sampler (geometric skip, the default, or keyed per sample)")
    ap.add_argument("--dec2", default="bp", choices=("bp", "bposd"),
                    help="phenl final-round decoder: BP, or BP+OSD-E(10) as the notebooks use")
    ap.add_argument("--num-cycles", type=int, default=13)
    return ap.parse_args()


def pauli_probs(eval_p):
    """EvalWER data branch arithmetic (src/Simulators.py:763-764): p = eval_p*3/2, [p/3]*3."""
    p = eval_p * 3 / 2
    return p / 3, p / 3, p / 3


def cpu_model() -> str:
    """The host CPU (lscpu's "Model name", from /proc/cpuinfo) for the cpu_baseline record."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.lower().startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def cpu_baseline(code, eval_p, max_iter, logical, budget_s):
    """Oracle (CPU restatement, fp64, host cores via OpenMP) on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker / baseline only

    # the CPUs this process may run on (the lease's allowance), not the host's logical CPU count;
    # OMP_NUM_THREADS (set by the GPU box's launcher to the lease's CPU share) caps it when present
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    cores = max(1, min(allowed, int(omp))) if omp and omp.isdigit() else max(1, allowed)
    px, py, pz = pauli_probs(eval_p)
    S = 32 * cores
    t0 = time.perf_counter()
    oracle.mc_run(code, px, py, pz, seed=SEED, shot_begin=0, shot_count=S, logical_mode=logical,
                  probs_x=eval_p, probs_z=eval_p, max_iter=max_iter, precision=64, nthreads=cores)
    dt = max(time.perf_counter() - t0, 1e-6)
    S2 = int(max(S, min(4_000_000, S * budget_s / dt)))
    t0 = time.perf_counter()
    r = oracle.mc_run(code, px, py, pz, seed=SEED, shot_begin=0, shot_count=S2, logical_mode=logical,
                      probs_x=eval_p, probs_z=eval_p, max_iter=max_iter, precision=64, nthreads=cores)
    dt = time.perf_counter() - t0
    return {"value": S2 / dt, "unit": "shots/s", "cores": cores, "kind": "port", "cpu_model": cpu_model(),
            "host_logical_cpus": os.cpu_count(), "affinity_cpus": allowed, "omp_num_threads": omp,
            "cores_rule": "min(len(os.sched_getaffinity(0)), OMP_NUM_THREADS): the CPUs the lease lets this "
                          "process use (the GPU box's launcher sets OMP_NUM_THREADS to the lease's CPU share)",
            "sample": f"{S2} shots of the same workload (shots 0..{S2 - 1}, same seed), oracle/qldpc_oracle.c "
                      f"fp64 with {cores} OpenMP threads, {dt:.1f} s; LER={r['failures'] / S2:.4g}",
            "note": "ORACLE PORT, not the reference: the reference's own CPU path (Python + the third-party ldpc "
                    "package, absent from this image and not installable offline) cannot run here; this is this "
                    "repository's C restatement of ldpc 0.1.x min-sum + the _single_run shot loop, compiled with "
                    "gcc -O3 and OpenMP (SURVEY.md 8d)"}


def kernel_name(dec):
    """Name of the fused MC kernel the decoder's geometry selects (as rocprofv3 reports it)."""
    g = dec.geometry()
    t = "float" if dec.precision == 32 else "double"
    if g["engine"] == 6:  # HBM-resident messages: staged pipeline around the per-lane decode kernel
        # decisions and syndromes as LDS ballot words for n + m <= 2048 (bp_hbm.hip hbm_xlds)
        xl = dec.graph.n + dec.graph.m <= 2048 and os.environ.get("QLDPC_HBM_XLDS", "1") != "0"
        return f"(anonymous namespace)::hdec_kernel<{t}, {'true' if xl else 'false'}> (engine 6, staged shot loop)"
    if g.get("kernel_id") in (11103, 31103, 40103):  # fp64 one-slot families (256 threads, NCH 3)
        return f"qldpc::rmc_kernel<double, 4, {g['vars_per_thread']}, {g['kernel_id']}, {g['degree3_slots']}, 256, 3>"
    if g.get("kernel_id") in (10103, 10203):  # fp64 one-word rows of 8, column degree 5 (kern_r_f64_m2s8.hip)
        return f"qldpc::rmc_kernel<double, 5, {g['vars_per_thread']}, {g['kernel_id']}, {g['degree3_slots']}, 256, 4>"
    mc = dec.graph.info()["max_col_deg"]
    dmax = 4 if mc <= 4 else (mc if g["engine"] == 3 and (mc <= 6 if dec.precision == 32 else mc == 5) else 8)
    nch = (max(1, dec.graph.info()["max_row_deg"]) * (4 if dec.precision == 32 else 8) + 15) // 16
    if g["engine"] == 3 and dec.precision == 64 and (dmax == 4 or (dmax == 5 and g["vars_per_thread"] <= 5)) \
            and g["threads"] <= 256 and 4 <= g["vars_per_thread"] <= 8 and nch in (3, 4) \
            and os.environ.get("QLDPC_F64W", "1") != "0":
        # fp64 family for <= 256-thread workgroups (engine id 103, launch bounds 256, rows of nch chunks)
        return f"qldpc::rmc_kernel<double, {dmax}, {g['vars_per_thread']}, 103, {g['degree3_slots']}, 256, {nch}>"
    if g["engine"] == 3 and dec.precision == 32 and dmax == 4 and 5 <= g["vars_per_thread"] <= 8 and nch == 2 \
            and os.environ.get("QLDPC_F32W", "1") != "0":
        # fp32 family with the compile-time 2-chunk check phase
        return f"qldpc::rmc_kernel<float, 4, {g['vars_per_thread']}, 3, {g['degree3_slots']}, 1024, 2>"
    if g["engine"] >= 3:
        return f"qldpc::rmc_kernel<{t}, {dmax}, {g['vars_per_thread']}, {g['engine']}, {g['degree3_slots']}>"
    return f"qldpc::smc_kernel<{t}, {dmax}, 1> (engine {g['engine']})"


def pmc_traffic(a):
    """HBM bytes per launch of the headline kernel, measured now on this build and config.

    Two rocprofv3 ``--pmc`` passes (FETCH_SIZE, WRITE_SIZE: separate runs, as gfx950 needs) over
    ``tools/prof_one.py``, which builds the same decoders and issues ONE launch of the same
    workload (code, p, shots, both sectors, precision, seed).  Runs as child processes BEFORE this
    process touches the GPU.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE x2,
    WRITE_SIZE as is; KB = 1024 B.  Returns a dict (bytes per launch, raw counters) or None.
    """
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    out = {}
    with tempfile.TemporaryDirectory(prefix="qldpc_pmc_", dir="/tmp") as td:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(td, counter)
            cmd = ["timeout", "-s", "KILL", "120", prof, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "p",
                   "--", sys.executable, os.path.join(ROOT, "tools", "prof_one.py"), a.code, str(a.p), str(a.shots), "0",
                   str(a.precision), a.logical, str(SEED), str(a.max_iter_ratio)]
            try:
                r = subprocess.run(cmd, cwd="/tmp", stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=150,
                                   env=dict(os.environ, TMPDIR="/tmp"))
            except (OSError, subprocess.SubprocessError):
                return None
            if r.returncode != 0:
                return None
            vals, kern = [], None
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for row in csv.DictReader(open(f)):
                    k = row.get("Kernel_Name", "")
                    # every kernel of the launch (the fused kernel, or the staged pipeline's kernels)
                    if row.get("Counter_Name") == counter and "at::native" not in k and "__amd_rocclr" not in k:
                        vals.append(float(row["Counter_Value"]))
                        if "mc_kernel" in k or "hdec_kernel" in k:
                            kern = k
            if not vals:
                return None
            out[counter] = sum(vals)
            out["kernel"] = kern
    # LDS bytes moved (SQ_INSTS_LDS_{LOAD,STORE,ATOMIC}_BANDWIDTH: units of 64 B, calibrated EXACT
    # against lds_calib's known byte counts, profiles/r04/calib/) and the bank-conflict share
    lds_cnt = ("SQ_INSTS_LDS_LOAD_BANDWIDTH", "SQ_INSTS_LDS_STORE_BANDWIDTH", "SQ_INSTS_LDS_ATOMIC_BANDWIDTH",
               "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE")
    lds = {}
    with tempfile.TemporaryDirectory(prefix="qldpc_pmc_", dir="/tmp") as td:
        cmd = ["timeout", "-s", "KILL", "120", prof, "--pmc", *lds_cnt, "--output-format", "csv", "-d", td, "-o", "p",
               "--", sys.executable, os.path.join(ROOT, "tools", "prof_one.py"), a.code, str(a.p), str(a.shots), "0",
               str(a.precision), a.logical, str(SEED), str(a.max_iter_ratio)]
        try:
            r = subprocess.run(cmd, cwd="/tmp", stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=150,
                               env=dict(os.environ, TMPDIR="/tmp"))
            if r.returncode == 0:
                for f in glob.glob(os.path.join(td, "**", "*counter_collection.csv"), recursive=True):
                    for row in csv.DictReader(open(f)):
                        k = row.get("Kernel_Name", "")
                        if ("mc_kernel" in k or "hdec_kernel" in k) and row.get("Counter_Name") in lds_cnt:
                            lds[row["Counter_Name"]] = lds.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        except (OSError, subprocess.SubprocessError):
            pass
    fetch_b = out["FETCH_SIZE"] * 2 * 1024
    write_b = out["WRITE_SIZE"] * 1024
    lds_out = None
    if all(k in lds for k in lds_cnt):
        lds_out = {"bytes": int(64 * (lds["SQ_INSTS_LDS_LOAD_BANDWIDTH"] + lds["SQ_INSTS_LDS_STORE_BANDWIDTH"]
                                      + lds["SQ_INSTS_LDS_ATOMIC_BANDWIDTH"])),
                   "load_bytes": int(64 * lds["SQ_INSTS_LDS_LOAD_BANDWIDTH"]),
                   "store_bytes": int(64 * lds["SQ_INSTS_LDS_STORE_BANDWIDTH"]),
                   "atomic_bytes": int(64 * lds["SQ_INSTS_LDS_ATOMIC_BANDWIDTH"]),
                   "bank_conflict_share": lds["SQ_LDS_BANK_CONFLICT"] / max(lds["SQ_LDS_IDX_ACTIVE"], 1.0),
                   "how": "rocprofv3 --pmc SQ_INSTS_LDS_{LOAD,STORE,ATOMIC}_BANDWIDTH SQ_LDS_BANK_CONFLICT "
                          "SQ_LDS_IDX_ACTIVE over one launch (tools/prof_one.py); x 64 B per unit, scale 1.000 "
                          "calibrated against tools/calib/lds_calib.hip's known byte counts"}
    return {"bytes": int(fetch_b + write_b), "fetch_bytes_x2": int(fetch_b), "write_bytes": int(write_b), "lds": lds_out,
            "fetch_size_kb_raw": out["FETCH_SIZE"], "write_size_kb_raw": out["WRITE_SIZE"], "kernel": out["kernel"],
            "how": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate runs) over tools/prof_one.py: one launch of this "
                   "workload; FETCH_SIZE x2 (gfx950), KB = 1024 B"}


def pmc_lds(args, kernel_substr):
    """LDS bytes moved per launch of one kernel, measured now: rocprofv3 --pmc
    SQ_INSTS_LDS_{LOAD,STORE,ATOMIC}_BANDWIDTH (units of 64 B, calibrated exact against
    tools/calib/lds_calib.hip, profiles/r04/calib/) + SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE over the
    child ``python <args>``, averaged over that kernel's dispatches.  Runs before this process touches
    the GPU.  Returns a dict or None."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    cnts = ("SQ_INSTS_LDS_LOAD_BANDWIDTH", "SQ_INSTS_LDS_STORE_BANDWIDTH", "SQ_INSTS_LDS_ATOMIC_BANDWIDTH",
            "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE")
    tot, disp = {}, set()
    with tempfile.TemporaryDirectory(prefix="qldpc_pmc_", dir="/tmp") as td:
        cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc", *cnts, "--output-format", "csv", "-d", td, "-o", "p", "--",
               sys.executable, *args]
        try:
            r = subprocess.run(cmd, cwd="/tmp", stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=180,
                               env=dict(os.environ, TMPDIR="/tmp"))
        except (OSError, subprocess.SubprocessError):
            return None
        if r.returncode != 0:
            return None
        for f in glob.glob(os.path.join(td, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if kernel_substr in row.get("Kernel_Name", "") and row.get("Counter_Name") in cnts:
                    tot[row["Counter_Name"]] = tot.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                    disp.add(row.get("Dispatch_Id"))
    if not all(k in tot for k in cnts) or not disp:
        return None
    nd = len(disp)
    return {"bytes": int(64 * (tot[cnts[0]] + tot[cnts[1]] + tot[cnts[2]]) / nd),
            "load_bytes": int(64 * tot[cnts[0]] / nd), "store_bytes": int(64 * tot[cnts[1]] / nd),
            "atomic_bytes": int(64 * tot[cnts[2]] / nd), "dispatches": nd,
            "bank_conflict_share": tot["SQ_LDS_BANK_CONFLICT"] / max(tot["SQ_LDS_IDX_ACTIVE"], 1.0),
            "how": f"rocprofv3 --pmc {' '.join(cnts)} over python {' '.join(os.path.basename(x) for x in args)}, "
                   f"x 64 B per unit (scale 1.000, profiles/r04/calib/), per dispatch of *{kernel_substr}*"}


def spawn_ranks(n):
    """``bench.py --gpus N`` without torchrun: N child ranks, one per GPU, started before this
    process touches any GPU (no exec from a GPU process); rank 0's JSON line is the output."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rcs = [p.wait() for p in procs]
    return max(abs(rc) for rc in rcs)


def st_kernel_roofline(torch, dec, Hst, p, B, bpe, bound, peak, dev, lds_pmc=None, peak_src=None):
    """The space-time decoder kernel alone (BASELINE config 5's dominant kernel): one decode_batch
    launch over B syndromes of i.i.d. errors at rate p on the stacked space-time graph, timed with
    HIP events on the stream it runs on (average of 3 launches after 1 warm-up).  Algorithmic bytes
    = bytes/edge-iteration x edges x the launch's summed iterations."""
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + 11)
    Hd = torch.zeros((Hst.m, Hst.n), dtype=torch.float32, device=dev)
    rows = torch.repeat_interleave(torch.arange(Hst.m, device=dev),
                                   torch.from_numpy(np.diff(Hst.row_ptr).astype(np.int64)).to(dev))
    Hd[rows, torch.from_numpy(np.asarray(Hst.col_idx, dtype=np.int64)).to(dev)] = 1.0
    e = (torch.rand((B, Hst.n), generator=g, device=dev) < p).to(torch.float32)
    synd = (torch.remainder(e @ Hd.t(), 2.0)).to(torch.uint8).contiguous()
    del e, Hd
    corr = torch.empty((B, Hst.n), dtype=torch.uint8, device=dev)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    conv = torch.empty(B, dtype=torch.uint8, device=dev)
    dec.decode_batch_device(synd, corr, iters, conv)
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps, it_sum = 3, 0
    ev0.record()
    for _ in range(reps):
        dec.decode_batch_device(synd, corr, iters, conv)
        it_sum += int(iters.sum().item()) if _ == reps - 1 else 0
    ev1.record()
    torch.cuda.synchronize(dev)
    ms = ev0.elapsed_time(ev1) / reps
    byts = bpe * it_sum * int(Hst.nnz)
    ach = byts / (ms / 1e3) / 1e9
    geo = dec.geometry()
    traffic = lds_pmc["bytes"] if (lds_pmc and bound == "lds") else None
    return {"bound": bound, "achieved": ach, "peak": peak, "unit": "GB/s", "frac": ach / peak, "traffic": traffic,
            "traffic_over_algorithmic": (traffic / byts) if traffic else None, "lds_pmc": lds_pmc,
            "peak_source": peak_src or ("HBM3E spec" if bound == "hbm" else "MI355X_MICROARCH.md aggregate"),
            "peak_guide_aggregate": LDS_PEAK_GBS if bound == "lds" else HBM_PEAK_GBS,
            "frac_guide_aggregate": ach / (LDS_PEAK_GBS if bound == "lds" else HBM_PEAK_GBS),
            "kernel": f"space-time decode_batch alone (engine {geo['engine']}, {geo['threads']} threads x "
                      f"{geo['vars_per_thread']} variables, {geo['lds_bytes']} B LDS)",
            "kernel_ms": ms, "bytes_per_launch": byts, "decodes_per_launch": B,
            "mean_iters": it_sum / B, "sample": f"{B} syndromes of i.i.d. errors at p={p} on the "
                                                f"{Hst.m}x{Hst.n} space-time graph"}


def phenl_main(a, torch, dist, world, rank, dev, st_pmc=None):
    """BASELINE config 5: CodeSimulator_Phenon_SpaceTime on the hgp_34_n1225_q3 stand-in (one line, not the headline).

    One step = ``--shots`` samples per GPU of ``num_rounds = (num_cycles-1)/num_rep + 1`` rounds
    (phenomenological noise p_data = q = eval_p, Pauli [eval_p/2]*3, src/Simulators_SpaceTime.py:1189-1216;
    decoder1 = space-time BP, decoder2 = BP, min-sum alpha=0.625, max_iter=int(n/10)).
    """
    from qldpc_fault_tolerance_amd import codes
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DevicePhenl

    name = a.code if a.code != "hgp_34_n1600" else "hgp_34_n1225_q3"
    code = codes.get_code(name)
    n, p, rep = code.N, a.p, a.num_rep
    R = int((a.num_cycles - 1) / rep + 1)
    mi = int(n / a.max_iter_ratio)
    hz, hx = code.csr("hz"), code.csr("hx")

    def st(H, m):
        return DeviceBP(codes.space_time_csr(H, rep), np.hstack([p * np.ones(n), p * np.ones(m)] * rep),
                        max_iter=mi, precision=a.precision, device=dev.index)

    soft = a.dec2 == "bposd"
    d2x = DeviceBP(hz, p * np.ones(n), max_iter=mi, precision=a.precision, device=dev.index, soft=soft)
    d2z = DeviceBP(hx, p * np.ones(n), max_iter=mi, precision=a.precision, device=dev.index, soft=soft)
    ph = DevicePhenl(code, st(code.hz, hz.m), st(code.hx, hx.m), d2x, d2z, num_rep=rep, max_batch=a.shots)
    if soft:
        from qldpc_fault_tolerance_amd.engine import DeviceOSD

        ph.set_final_osd(DeviceOSD(d2x.graph, p * np.ones(n), "osd_e", 10),
                         DeviceOSD(d2z.graph, p * np.ones(n), "osd_e", 10))
    S = int(a.shots)
    cnt = ph.new_counters()
    for i in range(a.warmup):
        ph.launch(p / 2, p / 2, p / 2, p, SEED + 3, (i * world + rank) * S, S, R, a.logical, cnt)
    torch.cuda.synchronize(dev)
    cnt.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        ph.launch(p / 2, p / 2, p / 2, p, SEED + 3, ((a.warmup + i) * world + rank) * S, S, R, a.logical, cnt)
    if world > 1:
        dist.all_reduce(cnt)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    w = cnt.cpu().numpy()
    shots, decodes, iters = int(w[0]), int(w[2] + w[3]), int(w[4] + w[5])
    # ST graph edges dominate: (num_rounds-1) ST decodes + 1 final decode per sector per sample
    E_st = int(codes.space_time_csr(code.hz, rep).nnz)
    E2 = int(hz.nnz)
    bpe = 16 if a.precision == 32 else 32
    frac_st = (R - 1) / R
    bytes_total = bpe * iters * (frac_st * E_st + (1 - frac_st) * E2)
    achieved = bytes_total / elapsed / 1e9 / world
    st_engine = ph.decoders[0].geometry()["engine"]
    bound, peak = ("hbm", HBM_PEAK_GBS) if st_engine == 6 else ("lds", LDS_PEAK_GBS)
    fam = mix_of_kernel(ph.decoders[0].geometry().get("kernel_id"), a.precision) if bound == "lds" else None
    peak_src = None
    if fam is not None:
        peak, peak_src = lds_ceiling(fam)
    stk = st_kernel_roofline(torch, ph.decoders[0], codes.space_time_csr(code.hz, rep), p, min(S, 65536), bpe, bound, peak,
                             dev, lds_pmc=st_pmc, peak_src=peak_src)
    out = {
        "metric": "phenomenological space-time samples/sec (BASELINE config 5; not the headline)",
        "value": shots / elapsed, "unit": "samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32" if a.precision == 32 else "f64",
        "data": f"synthetic: Philox phenomenological noise on the synthesized {name} stand-in",
        "config": {"workload": f"{name} CodeSimulator_Phenon_SpaceTime, num_rep={rep}, num_cycles={a.num_cycles} "
                               f"(num_rounds={R}), eval_p={p}, min-sum alpha=0.625, max_iter={mi}"
                               + (", decoder2 = BP+OSD-E(10)" if soft else ""),
                   "shots_per_gpu_step": S, "parallelism": f"sample-sharded x{world}"},
        "decodes_per_s": decodes / elapsed, "mean_iters_per_decode": iters / max(decodes, 1),
        "nonconverged_frac": int(w[6] + w[7]) / max(decodes, 1), "logical_error_rate": int(w[1]) / max(shots, 1),
        "roofline": stk,
        "pipeline_roofline": {"bound": bound, "achieved": achieved, "peak": peak, "unit": "GB/s",
                              "frac": achieved / peak,
                              "kernel": f"whole staged pipeline (wall clock, per GPU); space-time decoder engine {st_engine}"},
    }
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()


# VALU peak (MI355X_MICROARCH.md: 4 SIMD-32 per CU, a wave64 VALU op over 2 cycles): 256 CUs x 4 x 32
# 32-bit lane-ops per cycle at ~2.4 GHz
VALU_PEAK_GOPS = 256 * 4 * 32 * 2.4


def osd_kernel_roofline(torch, code, p, dx, dev, B=4096):
    """The GPU OSD kernel alone (BP+OSD's dominant kernel), on B syndromes whose soft-BP decodes did
    not converge at this p, timed with HIP events on the stream it runs on.  Bound: VALU.  Work
    model of the Gauss-Jordan elimination over GF(2) (dense upper bound): every one of the r pivots
    xors its row's remaining words into all m rows, on average W/2 64-bit words each = m * r * W / 2
    xors of 2 32-bit lane-ops; plus the OSD-E candidates: 2^w x ceil(r/64) words x (xor + popcount)."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceOSD

    import ctypes

    from qldpc_fault_tolerance_amd import _native

    n, m = code.N, code.hz.shape[0]
    soft = DeviceBP(code.hz, p * np.ones(n), max_iter=int(n / a_max_iter_ratio()), precision=64, device=dev.index, soft=True)
    osd = DeviceOSD(soft.graph, p * np.ones(n), "osd_e", 10)
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + 17)
    Hd = torch.from_numpy(code.hz.astype(np.float32)).to(dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    synd, post = [], []
    got = 0
    while got < B:  # keep only non-converged decodes (the ones BP+OSD sends to OSD)
        T = 4 * B
        e = (torch.rand((T, n), generator=g, device=dev) < p).to(torch.float32)
        sy = torch.remainder(e @ Hd.t(), 2.0).to(torch.uint8).contiguous()
        corr = torch.empty((T, n), dtype=torch.uint8, device=dev)
        it = torch.empty(T, dtype=torch.int32, device=dev)
        cv = torch.empty(T, dtype=torch.uint8, device=dev)
        ps = torch.empty((T, n), dtype=torch.float64, device=dev)
        _native.check(_native.lib().qldpc_bp_decode_batch_soft(
            soft.handle, ctypes.c_void_p(sy.data_ptr()), ctypes.c_void_p(corr.data_ptr()), ctypes.c_void_p(it.data_ptr()),
            ctypes.c_void_p(cv.data_ptr()), ctypes.c_void_p(ps.data_ptr()), T, st), "qldpc_bp_decode_batch_soft")
        keep = cv == 0
        synd.append(sy[keep])
        post.append(ps[keep])
        got += int(keep.sum().item())
        del e, corr, it, ps
    sd = torch.cat(synd)[:B].contiguous()
    pd = torch.cat(post)[:B].contiguous()
    del synd, post
    ow = torch.empty((B, n), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    osd.decode_device(sd, pd, None, None, None, ow)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    reps = 3
    for _ in range(reps):
        osd.decode_device(sd, pd, None, None, None, ow)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    from qldpc_fault_tolerance_amd.engine import HostOSD

    r = HostOSD(code.hz, p, "osd_e", 10).rank
    W = (n + 63) // 64
    w = min(10, n - r)
    ops = 2.0 * m * r * W / 2 + (1 << w) * ((r + 63) // 64) * 2.0
    ach = ops * B / (ms * 1e-3) / 1e9
    return {"bound": "valu", "achieved": ach, "peak": VALU_PEAK_GOPS, "unit": "Gop/s", "frac": ach / VALU_PEAK_GOPS,
            "traffic": None, "kernel": "osd_gpu_kernel (GPU OSD-E(10)) alone", "kernel_ms": ms, "syndromes": B,
            "us_per_syndrome_chip": ms * 1e3 / B, "ops_per_syndrome": ops, "rank": r,
            "model": "m*r*W/2 64-bit xors (dense Gauss-Jordan upper bound) + 2^w*ceil(r/64) candidate words; the "
                     "kernel is latency-bound on the pivot chain, so the fraction is small by construction"}


_MAX_ITER_RATIO = [10.0]


def a_max_iter_ratio():
    return _MAX_ITER_RATIO[0]


def bposd_main(a, torch, dist, world, rank, dev):
    """BP+OSD shot loop (not the headline): CodeSimulator_DataError with
    BPOSD_Decoder_Class(max_iter_ratio, "minimum_sum", 0.625, "osd_e", 10) sectors, as the notebooks
    build them.  One step = ``--shots`` shots per GPU through ``bposd_counts``: one fused engine-3
    launch per batch that captures the non-converged decodes on the device, the GPU OSD stage on
    those and the device re-check of their failures (no host round trips but the candidate count)."""
    from qldpc_fault_tolerance_amd import codes
    from qldpc_fault_tolerance_amd.decoders import BPOSD_Decoder_Class
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_DataError

    code = codes.get_code(a.code)
    p, S = a.p, int(a.shots)
    cls = BPOSD_Decoder_Class(a.max_iter_ratio, "minimum_sum", 0.625, "osd_e", 10, precision=a.precision,
                              device=dev.index)
    dx, dz = cls.GetDecoder({"h": code.hz, "p_data": p}), cls.GetDecoder({"h": code.hx, "p_data": p})
    sim = CodeSimulator_DataError(code, dx, dz, list(pauli_probs(p)), a.logical, seed=SEED + 5)
    for _ in range(a.warmup):
        sim.bposd_counts(S * world)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    fails = shots = osd_n = 0
    for _ in range(a.steps):
        f, c, o = sim.bposd_counts(S * world)
        fails, shots, osd_n = fails + f, shots + c, osd_n + o
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    mi = int(code.N / a.max_iter_ratio)
    _MAX_ITER_RATIO[0] = a.max_iter_ratio
    out = {
        "metric": "BP+OSD-E(10) shots/sec (SURVEY 8f rank 2; not the headline)", "value": shots / elapsed,
        "unit": "shots/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32" if a.precision == 32 else "f64",
        "data": f"synthetic: Philox-sampled depolarizing errors on {a.code}",
        "config": {"workload": f"{a.code} code-capacity BP+OSD shot loop, eval_p={p}, min-sum alpha=0.625, "
                               f"max_iter={mi}, osd_e order 10, eval_logical_type={a.logical}",
                   "shots_per_gpu_step": S, "parallelism": f"shot-sharded x{world}"},
        "osd_decodes": osd_n, "osd_frac_of_decodes": osd_n / max(1, 2 * shots),
        "logical_error_rate": fails / max(shots, 1),
        "roofline": osd_kernel_roofline(torch, code, p, None, dev) if world == 1 else None,
        "note": "wall clock of the device-resident BP+OSD loop: fused engine-3 MC capturing the decodes that reach "
                "max_iter (posteriors, syndrome, error), GPU OSD (osd_gpu_kernel) on those, device re-check of their "
                "residuals (qldpc_mc_set_osd)",
    }
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()


def native_comm_check(torch, dist, world, rank, dev, local, reduced):
    """After the timed steps (outside the timed region), all-reduce this rank's counters a second time
    through the engine's own C-ABI collective (qldpc_comm_init_rank + qldpc_comm_allreduce_counters,
    RCCL dlopen'ed by libqldpc_hip.so; rank 0's unique id broadcast over torch.distributed) and compare
    with torch.distributed's result.  Never fatal: a failure is reported in the JSON line."""
    if os.environ.get("QLDPC_NATIVE_COMM_CHECK", "1") == "0" or os.environ.get("QLDPC_DIST_BACKEND", "nccl") != "nccl":
        return None
    # every rank takes part in the broadcast and the final all-reduce whatever fails in between, so a
    # local failure cannot leave the other ranks waiting in a torch collective
    from qldpc_fault_tolerance_amd.parallel import NativeComm

    err, same = None, False
    uid = [None]
    if rank == 0:
        try:
            uid[0] = NativeComm.unique_id()
        except Exception as e:  # noqa: BLE001
            err = e
    dist.broadcast_object_list(uid, src=0)
    if uid[0] is not None:
        try:
            comm = NativeComm(dev.index, world, rank, uid[0])
            comm.allreduce_counters(local)
            torch.cuda.synchronize(dev)
            same = bool(torch.equal(local, reduced))
            comm.close()
        except Exception as e:  # noqa: BLE001
            err = e
    ok = torch.tensor([1 if same else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    out = {"native_allreduce_equals_torch": bool(ok.item()) if uid[0] is not None else None, "ranks": world,
           "how": "qldpc_comm_init_rank + qldpc_comm_allreduce_counters (C ABI, RCCL) on each rank's counters"}
    if err is not None:
        out["error"] = repr(err)[:300]
    return out


def native_comm_main(a, torch):
    """``--comm native``: ONE process drives ``--gpus`` GPUs through the C ABI only, as a host that
    binds ``libqldpc_hip.so`` without torch.distributed would: per GPU its own
    decoders and MC handle, ``qldpc_comm_init_all`` communicators, and per step one
    ``qldpc_mc_run_sharded`` call over ``--shots`` x N global shots (per-device blocks =
    parallel.shard_range, one host thread per device, one grouped RCCL all-reduce of the counters)."""
    from qldpc_fault_tolerance_amd import codes
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC, run_sharded
    from qldpc_fault_tolerance_amd.parallel import NativeComm

    if a.workload != "data":
        raise SystemExit("--comm native runs the data workload (config 2)")
    n = int(a.gpus)
    ndev = torch.cuda.device_count()
    if n > ndev:
        raise SystemExit(f"--comm native --gpus {n}: only {ndev} GPUs visible")
    code = codes.get_code(a.code)
    N = code.N
    mi = int(N / a.max_iter_ratio)
    p, S = a.p, int(a.shots)
    px, py, pz = pauli_probs(p)
    mcs = []
    for d in range(n):
        dx = DeviceBP(code.hz, p * np.ones(N), max_iter=mi, ms_scaling_factor=0.625, precision=a.precision, device=d)
        dz = DeviceBP(code.hx, p * np.ones(N), max_iter=mi, ms_scaling_factor=0.625, precision=a.precision, device=d,
                      vars_per_thread=dx.geometry()["vars_per_thread"])
        mcs.append(DeviceMC(code, dx, dz))
    comms = NativeComm.init_all(list(range(n))) if n > 1 else None
    for i in range(a.warmup):
        run_sharded(mcs, comms, px, py, pz, SEED, i * S * n, S * n, a.logical)
    for d in range(n):
        torch.cuda.synchronize(d)
    t0 = time.perf_counter()
    res = None
    for i in range(a.steps):
        r = run_sharded(mcs, comms, px, py, pz, SEED, (a.warmup + i) * S * n, S * n, a.logical)
        res = r if res is None else res.merge(r)
    elapsed = time.perf_counter() - t0
    if res.shots != S * n * a.steps:
        raise RuntimeError(f"counter mismatch: {res.shots} != {S} x {n} x {a.steps}")
    dec = sum(res.sector_decodes)
    emit({"metric": "BP-decoded shots/sec (node) on hgp_34_n1600 + % of HBM/LDS roofline", "value": res.shots / elapsed,
          "unit": "shots/s", "n_gpus": n, "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3,
          "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
          "dtype": "f32" if a.precision == 32 else "f64",
          "data": "synthetic: Philox-sampled depolarizing errors on the synthesized [[1600,64]] HGP stand-in",
          "config": {"workload": f"{a.code} code-capacity BP shot loop, eval_p={p}, min-sum alpha=0.625, max_iter={mi}, "
                                 f"eval_logical_type={a.logical}", "code": a.code, "p": p, "shots_per_gpu_step": S,
                     "parallelism": f"shot-sharded x{n}, one process, C-ABI qldpc_mc_run_sharded"
                                    + (" + qldpc_comm_init_all (RCCL)" if comms else "")},
          "decodes_per_s": dec / elapsed, "mean_iters_per_decode": sum(res.sector_iters) / max(dec, 1),
          "logical_error_rate": res.failures / max(res.shots, 1), "comm": "native"})


def circuit_kernel_roofline(torch, sim, g, dev, B):
    """The circuit loop's dominant kernel (the h1 round decode, 27 % of the r05 trace, profiles/r05/final/
    circuit_kernel_stats.csv) alone: decoder1's decode_batch over B round-0 syndromes of DEM samples,
    timed with HIP events on its stream (3 launches after 1 warm-up).  max_iter = int(N / 10) = 1 here,
    so the decode is the one-iteration first-min step kernel: it reads the precomputed
    per-edge magnitudes and never moves messages through LDS, so the bound is its HBM I/O (u8 syndrome
    in, u8 correction / int32 iterations / u8 flag out per syndrome) against 8 TB/s; the §8d message
    bytes of the same decodes (32 B per edge-iteration) are reported beside it."""
    dec1 = sim.decoder1_z.decoder
    R1, n1 = int(np.shape(g["h1"])[0]), int(np.shape(g["h1"])[1])
    E1 = int(np.asarray(g["h1"]).astype(bool).sum())
    det = sim._device().sample(sim.seed, 1 << 40, B)[:, :R1]  # round 0's detectors (no space correction yet)
    synd = torch.from_numpy(np.ascontiguousarray(det.astype(np.uint8))).to(dev)
    corr = torch.empty((B, n1), dtype=torch.uint8, device=dev)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    conv = torch.empty(B, dtype=torch.uint8, device=dev)
    dec1.decode_batch_device(synd, corr, iters, conv)
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    ev0.record()
    for _ in range(reps):
        dec1.decode_batch_device(synd, corr, iters, conv)
    ev1.record()
    torch.cuda.synchronize(dev)
    ms = ev0.elapsed_time(ev1) / reps
    io = B * (R1 + n1 + 4 + 1)
    it = int(iters.sum().item())
    ach = io / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "traffic": None, "kernel": f"decoder1 h1 decode_batch ({R1}x{n1}, max_iter {dec1.max_iter}: "
                                        f"{'one-iteration first-min step kernel' if dec1.max_iter == 1 else 'BP engine'})",
            "kernel_ms": ms, "bytes_per_launch": io, "decodes_per_launch": B,
            "algorithmic_message_bytes_GBs": 32 * E1 * it / (ms * 1e-3) / 1e9,
            "note": "HBM I/O per syndrome (R1 + n1 + 5 B) over the HIP-event time; the loop is launch- and "
                    "latency-bound at this graph size (DESIGN.md §4 circuit)"}


def circuit_main(a, torch, dist, world, rank, dev):
    """Circuit-level space-time (not the headline): the demo configuration of
    SpaceTimeDecodingDemo.ipynb cell 2 (hgp(ring_code(3), ring_code(3)), p = 1e-3, CX noise only,
    num_rep 3, num_cycles 13, ST_BP_Decoder_Circuit + ST_BPOSD_Decoder_Circuit OSD-E(10)) unless
    --p / --num-rep / --num-cycles say otherwise.  One step = ``--shots`` samples per GPU through
    ``qldpc_circ_launch`` (DEM sampling, the round loop, decoder2 BP+OSD on the host OSD stage)."""
    from qldpc_fault_tolerance_amd import codes
    from qldpc_fault_tolerance_amd.decoders import ST_BP_Decoder_Circuit, ST_BPOSD_Decoder_Circuit
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_Circuit_SpaceTime

    d = int(a.dem_d)
    ring = np.zeros((d, d), np.uint8)
    for i in range(d):
        ring[i, i] = ring[i, (i + 1) % d] = 1
    code = codes.hgp(ring, ring, name=f"toric_d{d}")
    p = a.p if a.p != DEFAULT_P else 1e-3
    if a.circuit_noise == "all":
        ep = {"p_i": p, "p_state_p": p, "p_m": p, "p_CX": p, "p_idling_gate": p}
    else:
        ep = {"p_i": 0.0, "p_state_p": 0.0, "p_m": 0.0, "p_CX": p, "p_idling_gate": 0.0}
    sim = CodeSimulator_Circuit_SpaceTime(code=code, p=p, num_cycles=a.num_cycles, num_rep=a.num_rep, error_params=ep,
                                          eval_logical_type="Z", seed=SEED + 7, sampler=a.sampler)
    sim._generate_circuit()
    sim._generate_circuit_graph()
    g = sim.circuit_graph
    mi = int(code.N / 10)
    sim.decoder1_z = ST_BP_Decoder_Circuit(g["h1"], g["channel_ps1"], mi, "minimum_sum", 0.625, device=dev.index)
    sim.decoder2_z = ST_BPOSD_Decoder_Circuit(g["h2"], g["channel_ps2"], mi, "minimum_sum", 0.625, "osd_e", 10,
                                              device=dev.index)
    S = int(a.shots)
    for _ in range(a.warmup):
        sim.fused_counts(S * world)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    shots = fails = 0
    for _ in range(a.steps):
        r = sim.fused_counts(S * world)
        shots, fails = shots + r.shots, fails + r.failures
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    from qldpc_fault_tolerance_amd.simulators import word_error_rate_per_cycle

    out = {"metric": "circuit-level space-time samples/sec (SURVEY 8f rank 4; not the headline)",
           "value": shots / elapsed, "unit": "samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f64", "data": "synthetic: Philox-sampled DEM mechanisms of the restated stim circuit",
           "config": {"workload": f"toric d{d} (hgp(ring_code({d}), ring_code({d}))), "
                                  + (f"p_CX={p}" if a.circuit_noise == "cx" else f"every noise source at p={p}")
                                  + f", num_rep={a.num_rep}, num_cycles={a.num_cycles}, BP (max_iter {mi}) rounds + "
                                    f"BP+OSD-E(10) final, {a.sampler} DEM sampler",
                      "samples_per_gpu_step": S, "dem_mechanisms": sim.dem.num_errors, "sampler": a.sampler,
                      "h1": list(np.shape(g["h1"])), "h2": list(np.shape(g["h2"])),
                      "parallelism": f"sample-sharded x{world}"},
           "logical_error_rate": fails / max(shots, 1),
           "wer_per_cycle": word_error_rate_per_cycle(fails, shots, code.K, a.num_cycles),
           "printed_reference_wer": 0.00019299501269032238 if (p == 1e-3 and a.num_cycles == 13 and a.num_rep == 3
                                                               and d == 3 and a.circuit_noise == "cx") else None,
           "roofline": circuit_kernel_roofline(torch, sim, g, dev, min(S, 65536))}
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()


_JSON_FD = None  # the real stdout: the JSON line is the only thing written there


def emit(out):
    line = (json.dumps(out) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, line)


def main():
    global _JSON_FD
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1 and a.comm == "torch":
        sys.exit(spawn_ranks(a.gpus))
    # library chatter on fd 1 (gloo's connection lines, runtime notices) goes to stderr, so rank 0's
    # stdout carries exactly one JSON line
    sys.stdout.flush()
    _JSON_FD = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    traffic = None
    st_pmc = None
    if a.workload == "data" and world == 1 and a.pmc_traffic and a.comm == "torch":
        traffic = pmc_traffic(a)  # child processes, before this process initialises the GPU
    if a.workload == "phenl" and world == 1 and a.pmc_traffic and a.comm == "torch":
        # the space-time decoder kernel alone, on the same syndromes st_kernel_roofline decodes
        name = a.code if a.code != "hgp_34_n1600" else "hgp_34_n1225_q3"
        st_pmc = pmc_lds([os.path.join(ROOT, "tools", "prof_st.py"), str(a.p), str(min(int(a.shots), 65536)),
                          str(a.precision), name, str(SEED + 11)], "rdec_kernel")
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; QLDPC_SHARE_GPU=1 lets ranks share the visible GPUs (multi-rank rehearsal on a
    # one-GPU box, with QLDPC_DIST_BACKEND=gloo since RCCL refuses two ranks on one device)
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % ndev if os.environ.get("QLDPC_SHARE_GPU") == "1" else local)
    torch.cuda.set_device(dev)
    if world > 1:
        backend = os.environ.get("QLDPC_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    if a.comm == "native":
        return native_comm_main(a, torch)
    if a.workload == "circuit":
        return circuit_main(a, torch, dist, world, rank, dev)
    if a.workload == "phenl":
        return phenl_main(a, torch, dist, world, rank, dev, st_pmc)
    if a.workload == "bposd":
        return bposd_main(a, torch, dist, world, rank, dev)

    from qldpc_fault_tolerance_amd import codes

    code = codes.get_code(a.code)
    r = time_data(a, a.precision, torch, dist, world, rank, dev)
    n = code.N
    max_iter = int(n / a.max_iter_ratio)
    p = a.p
    E = int(code.hz.sum())
    mh, nh = code.hz.shape
    # SURVEY.md §8d algorithmic bytes: 16 B (fp32) / 32 B (fp64) per edge-iteration of two-phase
    # flooding + per decode ceil(m/8)+ceil(n/8)+16 B of syndrome / decision / counters.
    bpe = 16 if a.precision == 32 else 32
    bytes_per_launch = (bpe * E * r["iters"] + r["decodes"] * ((mh + 7) // 8 + (nh + 7) // 8 + 16)) / (a.steps * world)
    achieved = bytes_per_launch / (r["kern_ms"] * 1e-3) / 1e9
    tb = traffic["bytes"] if traffic else None
    lds_t = traffic.get("lds") if traffic else None
    # engine 6 keeps the messages in HBM: the same algorithmic bytes are HBM bytes
    peak_src = None
    if r["engine"] == 6:
        bound, peak = "hbm", HBM_PEAK_GBS
    else:
        bound, peak = "lds", LDS_PEAK_GBS
        fam = mix_of_kernel(r.get("kernel_id"), a.precision)
        if fam is not None:
            peak, peak_src = lds_ceiling(fam)
    roof_traffic = (lds_t["bytes"] if lds_t else None) if bound == "lds" else tb
    peak_measured = None
    if bound == "lds" and peak_src and "measured" in peak_src:
        peak_measured = peak_src["measured"]["algorithmic_GBs"]
    out = {
        "metric": "BP-decoded shots/sec (node) on hgp_34_n1600 + % of HBM/LDS roofline",
        "value": r["value"],
        "unit": "shots/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": r["elapsed"] / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if a.precision == 32 else "f64",
        "data": "synthetic: Philox-sampled depolarizing errors on the synthesized [[1600,64]] HGP stand-in "
                "(the reference's hgp_34_n1600.pkl is missing; DESIGN.md)",
        "config": {"workload": f"{a.code} code-capacity BP shot loop, eval_p={p}, min-sum alpha=0.625, "
                               f"max_iter={max_iter}, eval_logical_type={a.logical}, "
                               + ("float64 messages = ldpc's arithmetic" if a.precision == 64 else
                                  "float32 fast mode (NOT the reference arithmetic)"),
                   "code": a.code, "p": p, "shots_per_gpu_step": a.shots, "max_iter": max_iter,
                   "decodes_per_shot": int(a.logical != "Z") + int(a.logical != "X"),
                   "parallelism": f"shot-sharded x{world}"},
        "decodes_per_s": r["decodes"] / r["elapsed"],
        "mean_iters_per_decode": r["iters"] / max(r["decodes"], 1),
        "nonconverged_frac": r["nonconv"] / max(r["decodes"], 1),
        "logical_error_rate": r["failures"] / max(r["shots"], 1),
        "comm_check": r.get("comm_check"),
        "roofline": {"bound": bound, "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "traffic": roof_traffic,
                     "traffic_over_algorithmic": (roof_traffic / bytes_per_launch) if roof_traffic else None,
                     "peak_source": (peak_src if (bound == "lds" and peak != LDS_PEAK_GBS) else
                                     "MI355X_MICROARCH.md aggregate" if bound == "lds" else "HBM3E spec"),
                     "peak_measured": peak_measured,
                     "frac_measured": (achieved / peak_measured) if peak_measured else None,
                     "peak_guide_aggregate": LDS_PEAK_GBS if bound == "lds" else HBM_PEAK_GBS,
                     "frac_guide_aggregate": achieved / (LDS_PEAK_GBS if bound == "lds" else HBM_PEAK_GBS),
                     "lds_pmc": lds_t,
                     "kernel": r["kernel"], "kernel_ms": r["kern_ms"],
                     "bytes_per_launch": bytes_per_launch,
                     # HBM carries only the edge tables (L2-resident) and the counters
                     "hbm": {"achieved": (tb / (r["kern_ms"] * 1e-3) / 1e9) if tb else None,
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "pmc": traffic}},
    }
    if world == 1 and a.precision == 64 and a.fp32_line:
        # fp32 fast mode on the same workload: reported beside the headline, never as `value`
        r32 = time_data(a, 32, torch, dist, world, rank, dev)
        # on the headline's basis: the same algorithmic bytes (16 B per edge-iteration in fp32) over the
        # kernel's HIP-event time, against its own family's LDS row-mix ceiling
        ach32 = (16 * E * r32["iters"] / a.steps + r32["decodes"] / a.steps * ((mh + 7) // 8 + (nh + 7) // 8 + 16)) \
            / (r32["kern_ms"] * 1e-3) / 1e9
        fam32 = mix_of_kernel(r32.get("kernel_id"), 32, E // mh if E % mh == 0 else None)
        peak32, src32 = lds_ceiling(fam32) if fam32 else (LDS_PEAK_GBS, "MI355X_MICROARCH.md aggregate")
        out["fp32_fast_mode"] = {
            "value": r32["value"], "unit": "shots/s", "ms_per_step": r32["elapsed"] / a.steps * 1e3,
            "kernel": r32["kernel"], "kernel_ms": r32["kern_ms"],
            "roofline": {"bound": "lds", "achieved": ach32, "peak": peak32, "unit": "GB/s", "frac": ach32 / peak32,
                         "peak_source": src32, "frac_guide_aggregate": ach32 / LDS_PEAK_GBS},
            "roofline_frac": ach32 / peak32,
            "logical_error_rate": r32["failures"] / max(r32["shots"], 1),
            "note": "float32 messages: NOT ldpc's float64 arithmetic (decoded-vector agreement with fp64 is "
                    "measured in tests/test_gpu_agreement.py)"}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(code, p, max_iter, a.logical, a.cpu_seconds)
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()


def time_data(a, precision, torch, dist, world, rank, dev):
    """BASELINE config 2: W warmup launches, then K timed launches of ``--shots`` shots per GPU
    bracketed by barrier + synchronize, max over ranks; HIP events on the launch stream time the
    kernel.  Returns the all-reduced counters and the timings."""
    from qldpc_fault_tolerance_amd import codes
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC

    code = codes.get_code(a.code)
    n = code.N
    max_iter = int(n / a.max_iter_ratio)
    p = a.p
    px, py, pz = pauli_probs(p)
    need_x, need_z = a.logical != "Z", a.logical != "X"
    # decoders as EvalWER builds them: p_data = eval_p on hz (X errors) and hx (Z errors)
    dx = DeviceBP(code.hz, p * np.ones(n), max_iter=max_iter, bp_method="minimum_sum", ms_scaling_factor=0.625,
                  precision=precision, device=dev.index) if need_x else None
    # the Z-sector decoder takes the X sector's geometry (one fused kernel serves both)
    vpl = dx.geometry()["vars_per_thread"] if dx is not None and not os.environ.get("QLDPC_TB") else 0
    dz = DeviceBP(code.hx, p * np.ones(n), max_iter=max_iter, bp_method="minimum_sum", ms_scaling_factor=0.625,
                  precision=precision, device=dev.index, vars_per_thread=vpl) if need_z else None
    mc = DeviceMC(code, dx, dz)
    S = int(a.shots)
    stream = torch.cuda.current_stream(dev)
    cnt = mc.new_counters()

    def step(i):
        # global shot blocks indexed by (step, rank): shot ranges never overlap across ranks
        mc.launch(px, py, pz, SEED, (i * world + rank) * S, S, a.logical, cnt)

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    cnt.zero_()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for i in range(a.steps):
        ev[i][0].record(stream)
        step(a.warmup + i)
        ev[i][1].record(stream)
    local = cnt.clone() if world > 1 else None  # this rank's counters (for the C-ABI cross-check)
    if world > 1:
        dist.all_reduce(cnt)  # shots, failures, iterations, non-converged, histogram
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    comm_check = native_comm_check(torch, dist, world, rank, dev, local, cnt) if world > 1 and precision == a.precision \
        else None
    w = cnt.cpu().numpy()
    shots = int(w[0])
    if shots != S * a.steps * world:
        raise RuntimeError(f"counter mismatch: {shots} shots != {S} x {a.steps} x {world}")
    return {"value": shots / elapsed, "elapsed": elapsed, "kern_ms": kern_ms, "shots": shots, "failures": int(w[1]),
            "decodes": int(w[2] + w[3]), "iters": int(w[4] + w[5]), "nonconv": int(w[6] + w[7]),
            "kernel": kernel_name(dx or dz), "engine": (dx or dz).geometry()["engine"],
            "kernel_id": (dx or dz).geometry().get("kernel_id"), "comm_check": comm_check}


if __name__ == "__main__":
    main()
