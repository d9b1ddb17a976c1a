#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: GiB/s of device-resident AES-128-GCM TLS record
decrypt (tls1_enc(s, 0) / EVP_AEAD_CTX_open per record), 16 KiB records, batch
64 Ki records per GPU (configs[1]; configs[4] = the same per-GPU batch on 8 GPUs).

One step = one tlsgpu_open_batch over the whole resident batch (64 Ki records,
1 GiB of ciphertext in HBM -> 1 GiB of plaintext in HBM + per-record status).
Inputs are synthetic (counter-SplitMix64 plaintexts, 1024 sessions x 64 records,
1/1024 records tampered), sealed on the device beforehand by the validated
sealer; the first step's outputs are verified before the warm-up steps (so the
GPU is busy up to the timed region) and the last timed step's after it.  Before
the W warm-up steps an untimed settle (--settle-ms, default 100 ms of
back-to-back steps) lets the GPU clock leave the dip a fresh sustained load
causes, so the K timed steps measure the steady state.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config B|C|D]
                  [--sessions S] [--interleave] [--mode device|host|wire|copy]
                  [--split group|ranks] [--devices 0,1,...]
  N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
       runs config E (configs[4]) through the C ABI's own batch split by
       default: rank 0 drives a tlsgpu_group of N member GPUs (group.cpp), the
       other ranks only join the barrier.  --split ranks: one rank per GPU,
       records split by rank, each rank its own engine.  Either way no
       collective on the data path; gloo only carries the barrier and the
       max-over-ranks of the timing.

Prints ONE JSON line (rank 0).  `roofline.achieved` = algorithmic bytes per
launch / average launch time from HIP events on the engine stream;
`cpu_baseline` = the reference LibreSSL EVP_AEAD_CTX_open (oracle/_ref/libref.so,
compiled from the reference sources) on a bounded sample on this host.
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

METRIC = "GiB/s device-resident AES-128-GCM TLS record decrypt, 16KiB recs, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)

CONFIGS = {
    # name: (kind, records per GPU, sessions per GPU, record_len or None(zipf), seed, op)
    "B": ("aes-128-gcm", 65536, 1024, 16384, 0x5EED0001, "open"),
    "C": ("chacha20-poly1305", 1 << 20, 4096, 1400, 0x5EED0002, "seal+open"),
    "D": ("aes-256-gcm", 1 << 18, 1024, None, 0x5EED0003, "open"),
    # configs[4]: ONE batch of 512 Ki x 16 KiB records (8,192 sessions) split
    # across 8 GPUs; GPU r opens shard r (records [64 Ki r, 64 Ki (r + 1)))
    "E": ("aes-128-gcm", 65536, 1024, 16384, 0x5EED0004, "open"),
}
E_GPUS = 8   # config E's batch is defined over 8 shards


def algo_bytes_per_record(kind_name: str, length: int, op: str, read_only: bool = False) -> int:
    """read explicit nonce + ct + tag + 32-B descriptor, write pt + status."""
    eiv = 8 if "gcm" in kind_name else 0
    rd = eiv + length + 16 + 32
    wr = length + 4
    return rd if read_only else rd + wr


def main_kernel(kind_name: str, op: str, short_records: bool = False, short_runs: bool = False,
                records: int = 1 << 30) -> str:
    """Name of the step's dominant kernel as rocprofv3 lists it: the queue kernel's
    pack variant runs when the batch has records of <= 62 blocks,
    the per-wave-session kernel when session runs average < 12 records (§4.1d)."""
    import talos_amd as ta
    if "gcm" not in kind_name:   # the LDS-staged TLS kernel; C = seal + open
        return "tg::chacha_tls_kernel" if op == "seal+open" else \
            f"tg::chacha_tls_kernel<{'true' if op == 'seal' else 'false'}>"
    rounds = 10 if "128" in kind_name else 14
    seal = "true" if op != "open" else "false"
    impl = ta.get_gcm_impl()
    if impl == "split" or (impl == "auto" and records <= 512):  # small batch: <= 2 records per CU
        return f"tg::gcm_raw_kernel<{seal}, {rounds}, true>"
    impl = "queue" if impl == "auto" else impl
    pws = os.environ.get("TLSGPU_PWS", "")
    if impl == "queue" and (pws == "1" or (pws != "0" and short_runs)):
        return f"tg::gcm_pw_kernel<{seal}, {rounds}>"
    pack = ", true" if short_records and os.environ.get("TLSGPU_PACK", "1") != "0" else ", false"
    return {"queue": f"tg::gcm_hy_kernel<{seal}, {rounds}, 1024, 0, 2{pack}, 0>",
            "hybrid": f"tg::gcm_hy_kernel<{seal}, {rounds}, 512, 4, 4, false>",
            "bitslice": f"tg::gcm_hy_kernel<{seal}, {rounds}, 512, 8, 4, false>",
            "fused": f"tg::gcm_fused_kernel<{seal}, {rounds}>",
            "ttable": f"tg::gcm_batch_kernel<{seal}, false, {rounds}>"}[impl]


def host_cpus() -> tuple[int, int, str, str]:
    """(threads usable by this process, visible cores, CPU model, what limits it).
    Usable = the affinity set, capped by the cgroup CPU quota (cpu.max) when one
    is set: on the GPU box the process's share is a quota, not a cpuset."""
    visible = len(os.sched_getaffinity(0))
    usable, why = visible, "sched_getaffinity"
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
            if quota < usable:
                usable, why = quota, f"cgroup cpu.max quota ({q}/{period})"
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, visible, model, why


def cpu_baseline(kind_name: str, rec_len, op: str, note: str = "") -> dict | None:
    """Reference LibreSSL EVP_AEAD_CTX_open/seal (oracle/_ref/libref.so) on every
    core this process may use; rec_len is an int or an array of record lengths
    (the Zipf mix itself, passed to cpubench as a lengths file)."""
    # the reference build links LibreSSL's x86-64 AES-NI and PCLMUL GHASH
    # assembly (oracle/Makefile); its ChaCha20 and Poly1305 are the portable C
    impl = ("AES-NI + PCLMUL GHASH asm" if "gcm" in kind_name
            else "portable C chacha.c + poly1305-donna")
    try:
        import tempfile
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        if not (os.path.exists(pyoracle.LIBREF) and os.path.exists(pyoracle.CPUBENCH)):
            return None
        threads, visible, model, why = host_cpus()
        secs = max(1.0, 20.0 / threads)   # ~20 s of CPU work in total
        if np.ndim(rec_len):
            lens = np.asarray(rec_len, dtype=np.uint32)
            nrec = len(lens)
            with tempfile.NamedTemporaryFile(suffix=".u32", delete=False) as f:
                f.write(lens.tobytes())
                arg = "@" + f.name
            what = f"{nrec} records of the workload's own length mix (mean {lens.mean():.0f} B)"
        else:
            nrec = max(threads * 16, 1024)
            arg, what = rec_len, f"{nrec} x {rec_len}-B records"
        r = pyoracle.run_cpubench(kind_name, "both" if op == "seal+open" else op, arg, nrec,
                                  threads, secs)
        if isinstance(arg, str):
            os.unlink(arg[1:])
        return {"value": round(r["gib_per_s"], 3), "unit": "GiB/s", "cores": threads,
                "kind": "reference",
                "host": f"{model}; {threads} threads = {why}, {visible} cores visible",
                "sample": f"LibreSSL 2.4.1 EVP_AEAD_CTX_{op} ({impl}) over {what}{note}, "
                          f"{threads} pthreads x {secs:.1f}s ({r['records']} records timed), "
                          f"oracle/_ref/libref.so"}
    except Exception as exc:  # baseline is reported, never fatal
        return {"value": None, "error": str(exc)[:200]}


def load_traffic(config: str, kernel: str):
    """PMC-measured HBM bytes per launch of `kernel`, if a profile of that same
    kernel was committed (scripts/pmc_summary.py): the L2's memory-side read
    requests by size (TCC_EA0_RDREQ_128B/64B/32B) + WRITE_SIZE when that pass
    exists, else FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md §HBM)."""
    p = os.path.join(ROOT, "profiles", f"pmc_config{config}.json")
    if os.path.exists(p):
        try:
            d = json.load(open(p))
            if kernel in d.get("kernel", ""):
                return (d.get("hbm_bytes_per_launch_by_request_size") or
                        d.get("hbm_bytes_per_launch")), os.path.relpath(p, ROOT)
        except Exception:
            return None, None
    return None, None


# Measured pipe rates (tools/ubench.hip, profiles/r03a_ubench.jsonl, 16 waves
# per CU): CU cycles per ds_read_b32 in dependent lookup chains and per
# conflict-free ds_read_b128 — the LDS issue the T-table GCM loop is bound by.
LDS_B32_CYC, LDS_B128_CYC = 2.32, 4.96
AES_LOOKUPS = {10: 138, 14: 202}   # ds_read_b32 per 64-block step (TLS counter shortcut)
GHASH_B128 = 16                    # ds_read_b128 per 64-block Horner step (byte-position table)


def pmc_profile(config: str, kernel: str):
    p = os.path.join(ROOT, "profiles", f"pmc_config{config}.json")
    try:
        d = json.load(open(p))
        return d if kernel in d.get("kernel", "") else None
    except (OSError, ValueError):
        return None


def compute_roofline(kind_name: str, lengths, per_launch_s: float, prof, cus: int) -> dict:
    """The binding on-chip pipe: for AES-GCM the LDS, priced
    with the measured rates above — compute_ceiling = the payload rate at which
    this launch's algorithmic lookups would keep every CU's LDS busy at those
    rates, at the clock the kernel ran under PMC (GRBM_GUI_ACTIVE / 8 XCDs /
    duration, profiles/pmc_config*.json).  Plus the PMC pipe-busy fractions."""
    out = {}
    clock = 2.05e9
    c = (prof or {}).get("counters_per_launch_mean", {})
    dur = (prof or {}).get("mean_duration_ns_profiled")
    if c.get("GRBM_GUI_ACTIVE") and dur:
        clock = c["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e-9)
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        if c.get("SQ_LDS_IDX_ACTIVE"):
            out["pmc_lds_busy"] = round(c["SQ_LDS_IDX_ACTIVE"] / (cus * cyc), 3)
        if c.get("SQ_INSTS_VALU"):   # 2 cycles per wave64 VALU op on a SIMD-32 (lower bound)
            out["pmc_valu_busy_lb"] = round(c["SQ_INSTS_VALU"] * 2 / (4 * cus * cyc), 3)
        out["pmc_clock_ghz"] = round(clock / 1e9, 3)
    if "gcm" in kind_name:
        rounds = 10 if "128" in kind_name else 14
        steps = sum((int(l) + 16 + 15) // 16 / 64.0 for l in lengths)   # data + AAD + lengths blocks
        lds_cyc = steps * (AES_LOOKUPS[rounds] * LDS_B32_CYC + GHASH_B128 * LDS_B128_CYC) / cus
        ceiling = float(sum(int(l) for l in lengths)) / (lds_cyc / clock) / GIB
        out.update({"compute_bound": "lds", "compute_ceiling_GiBps": round(ceiling, 1),
                    "compute_model": f"{AES_LOOKUPS[rounds]} ds_read_b32 x {LDS_B32_CYC} + "
                                     f"{GHASH_B128} ds_read_b128 x {LDS_B128_CYC} CU-cycles per "
                                     f"64-block step at {clock / 1e9:.2f} GHz"})
    else:
        out["compute_bound"] = "valu"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # 30: the GPU reaches its working clock after ~30 ms of back-to-back steps
    # (B: warm-up 3 / 10 / 30 / 60 / 100 -> 953 / 1,028 / 1,065 / 1,053 / 1,069
    # GiB/s; profiles/r05ag_bench_warm_start.txt); a warm-up is untimed
    ap.add_argument("--warmup", type=int, default=30)
    # untimed settle before the W warm-up steps: back-to-back steps until the
    # GPU's clock has left the dip a fresh sustained load causes (2.07 -> 1.61
    # GHz, back to ~2.3 GHz after ~30 ms; profiles/r05ag_bench_warm_start.txt:
    # W = 3 / 10 / 30 / 60 / 100 -> 953 / 1,028 / 1,065 / 1,053 / 1,069 GiB/s),
    # so that K timed steps measure the steady state whatever W the caller picks
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="untimed back-to-back steps for at least this long before the "
                         "warm-up (0: none)")
    ap.add_argument("--config", default="B", choices=sorted(CONFIGS))
    ap.add_argument("--records", type=int, default=0, help="override records per GPU")
    ap.add_argument("--sessions", type=int, default=0,
                    help="override sessions per GPU (SURVEY.md §8d sensitivity: 1 .. #records)")
    ap.add_argument("--slot-align", type=int, default=16,
                    help="alignment of every record's plaintext and ciphertext slot in the "
                         "device buffers (default 16; 128 = each record on its own cache lines, "
                         "a measurement option: the golden digests use 16)")
    ap.add_argument("--interleave", action="store_true",
                    help="deal records to sessions round-robin (a many-connection server "
                         "batch) instead of grouping each session's records")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-hints", action="store_true",
                    help="do not state the batch-shape hints (tlsgpu_sessions_hint) the "
                         "workload's lengths and session order imply")
    ap.add_argument("--host-streams", type=int, default=0, help="host mode: pipeline streams")
    ap.add_argument("--host-chunk-mib", type=int, default=0, help="host mode: chunk size")
    ap.add_argument("--split", default=None, choices=["group", "ranks"],
                    help="multi-GPU batch split: group = the C ABI's own split "
                         "(tlsgpu_group_open_batch: one process drives every member GPU; the "
                         "default for N > 1), ranks = one torch.distributed rank per GPU, each "
                         "with its own engine")
    ap.add_argument("--devices", default="",
                    help="group split: comma-separated device ids (default 0..N-1); "
                         "'0,0' rehearses a two-member group on one GPU")
    ap.add_argument("--mode", default="device", choices=["device", "host", "wire", "copy", "pcie"],
                    help="host: pinned host buffers + H2D/D2H overlap (PCIe-inclusive rate); "
                         "wire: raw TLS wire streams through tlsgpu_open_wire (framing + "
                         "in-place open, SURVEY.md §8f-1); copy: the box's achievable "
                         "device-to-device copy bandwidth (hipMemcpy, 1 GiB)")
    args = ap.parse_args()

    import talos_amd as ta
    from talos_amd.dist import ControlPlane, device_for, env_rank, shard_by_bytes
    from talos_amd.workload import Workload, zipf_lengths

    world, rank, local = env_rank()
    if choose_split(args.split, world, args.devices, args.gpus) == "group" and args.mode == "device":
        return group_mode(args, world, rank)
    ta.load_library()
    eng = ta.Engine(device_for(local, ta.device_count()))  # first GPU runtime user
    if args.mode == "copy":
        return copy_mode(args, eng)
    if args.mode == "pcie":
        return pcie_mode(args, eng)
    cp = ControlPlane(world)   # gloo control plane: barrier + max over ranks only

    # N > 1 GPUs run BASELINE configs[4] (config E) unless a config is named:
    # the headline metric's multi-GPU line
    if world > 1 and args.config == "B" and not args.records and not args.sessions:
        args.config = "E"
    kind_name, per_gpu, sessions, rec_len, seed, op = CONFIGS[args.config]
    if args.records:
        per_gpu = args.records
        sessions = max(1, min(sessions, per_gpu // 16))
    if args.sessions:
        sessions = min(args.sessions, per_gpu)
    kind = ta.AEAD_NAMES[kind_name]
    # weak scaling: ONE global batch of shards x per_gpu records (config E: 8
    # shards whatever N is, GPU r opens shard r; the others: N shards); rank r
    # owns a contiguous equal-byte slice, no data-path
    # collective.  Every rank builds its slice with global record indices
    # (talos_amd.workload), so shard r is the same bytes at any N and
    # tests/golden/batch_digests.json E_shard<r> pins it.
    shards = max(E_GPUS, world) if args.config == "E" else world
    glob = (np.full(shards * per_gpu, rec_len, dtype=np.int64) if rec_len else
            zipf_lengths(shards * per_gpu, seed))
    lo, hi = shard_by_bytes(glob, shards, rank)
    lengths = None if rec_len else glob[lo:hi]
    wl = Workload(eng, kind, shards * per_gpu, shards * sessions, seed, lengths=lengths,
                  slot_align=args.slot_align,
                  record_len=rec_len or 0,
                  tamper_every=1024 if op == "open" and args.mode != "wire" else 0,
                  interleave=args.interleave, shard=(lo, hi))
    total_len = int(wl.lengths.sum())
    # what the caller that built the batch knows about its shape (no short GCM
    # records / long session runs): the engine then skips the launches of the
    # kernel variants the device would not select (tlsgpu.h tlsgpu_sessions_hint)
    # descriptor lengths: fragments for an open, plaintexts for a seal
    desc_len = wl.lengths + (ta.EXPLICIT_NONCE_LEN[kind] + ta.TAG_LEN if op == "open" else 0)
    hints = 0 if args.no_hints else ta.batch_hints(desc_len, wl.session, seal=op != "open")
    wl.table.hint(hints)
    args.hints = hints
    if args.mode == "host":
        return host_mode(args, eng, wl, kind_name, total_len)
    if args.mode == "wire":
        return wire_mode(args, eng, wl, kind_name, total_len)

    def step(stream=None):
        if op == "open":
            wl.open(stream)
        else:
            wl.seal(stream)
            wl.open(stream)

    # the first step's outputs are verified before the warm-up, not after it:
    # the verification's host round trips leave the GPU idle for tens of ms,
    # and the timed region must start at the working clock the warm-up reached
    # (profiles/r05ag_bench_warm_start.txt)
    step()
    eng.sync()
    wl.verify_open()
    settled = settle(step, eng.sync, args.settle_ms)
    for _ in range(max(1, args.warmup)):
        step()

    def barrier():
        eng.sync()
        cp.barrier()

    phase = bool(os.environ.get("TLSGPU_PHASE_STATS"))
    if phase:
        ta.debug_phase_stats(eng, reset=True)
    ev0, ev1 = ta.Event(eng), ta.Event(eng)
    barrier()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    eng.sync()
    t1 = time.perf_counter()
    dev_ms = ev0.elapsed_ms(ev1)
    wall_ms = (t1 - t0) * 1e3
    if phase:  # diagnostic: per-phase shader cycles of the hybrid kernel, per step
        st = ta.debug_phase_stats(eng, reset=True)
        names = {1: "bs-aes", 2: "bs-consume", 3: "bs-finish", 4: "bs-barrier", 5: "tables",
                 6: "tt-switch",
                 9: "tt-x4", 10: "tt-rest", 11: "tt-finish", 12: "tt-barrier",
                 13: "pack", 14: "recs/pack", 15: "plan"}
        for i, nm in names.items():
            if st[2 * i + 1]:
                print(f"phase {nm:11s} cycles/step {st[2*i]/args.steps:14.0f} events/step "
                      f"{st[2*i+1]/args.steps:9.0f} cycles/event {st[2*i]/st[2*i+1]:9.0f}",
                      file=sys.stderr)
    barrier()
    wl.verify_open()

    elapsed_s, wall_s = cp.max([dev_ms / 1e3, wall_ms / 1e3])
    total_payload = cp.sum([float(total_len)])[0]

    payload = total_payload * args.steps                      # plaintext bytes, all ranks
    value = payload / elapsed_s / GIB
    per_launch_s = dev_ms / 1e3 / args.steps / (2 if op == "seal+open" else 1)
    algo = sum(algo_bytes_per_record(kind_name, int(l), op) for l in
               ([rec_len] * wl.n if lengths is None else lengths.tolist()))
    achieved = algo / per_launch_s / 1e9
    algo_rd = sum(algo_bytes_per_record(kind_name, int(l), op, True) for l in
                  ([rec_len] * wl.n if lengths is None else lengths.tolist()))
    # session runs of the batch (prep-pass selection, tlsgpu_internal.h pws_selected)
    runs = per_gpu if args.interleave and sessions > 1 else min(sessions, per_gpu)
    kernel = main_kernel(kind_name, op, CONFIGS[args.config][3] is None, runs * 12 > per_gpu, wl.n)
    prof_cfg = "B" if args.config == "E" else args.config   # same kernel, same per-GPU batch
    traffic, traffic_src = load_traffic(prof_cfg, kernel)
    comp = compute_roofline(kind_name, [rec_len] * wl.n if lengths is None else lengths.tolist(),
                            per_launch_s, pmc_profile(prof_cfg, kernel), eng.num_cus)
    if "compute_ceiling_GiBps" in comp:
        comp["compute_frac"] = round(value / world / comp["compute_ceiling_GiBps"], 4)

    line = {
        "metric": METRIC if args.config in ("B", "E") else
        f"GiB/s device-resident {kind_name} TLS record {op} (config {args.config})",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle": settled,
        "ms_per_step": round(elapsed_s * 1e3 / args.steps, 4),
        "wall_ms_per_step": round(wall_s * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter-SplitMix64 plaintexts sealed on device; 1/1024 tampered)"
        if op == "open" else "synthetic (counter-SplitMix64 plaintexts)",
        "config": {"workload": (f"config {args.config}: " if args.config in ("B", "E") else "") +
                               f"{kind_name} TLS 1.2 record {op}, "
                               f"{'16 KiB' if rec_len == 16384 else (str(rec_len) + ' B' if rec_len else 'Zipf 64 B-16 KiB')}"
                               f" records, {per_gpu} records/GPU, device-resident" +
                               (f"; shards 0..{world - 1} of one {shards * per_gpu}-record batch "
                                f"(seed {seed:#x}, {shards * sessions} sessions)"
                                if args.config == "E" else ""),
                   "records_per_gpu": per_gpu, "sessions_per_gpu": sessions,
                   "session_order": "interleaved" if args.interleave else "grouped",
                   "slot_align": args.slot_align,
                   "gcm_impl": ta.get_gcm_impl() if "gcm" in kind_name else None,
                   "batch_hints": args.hints,
                   "payload_bytes_per_gpu": total_len, "parallelism": f"batch split x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "algorithmic_bytes_per_launch": algo,
                     # north_star prices the "HBM-read roofline": the read half alone
                     "read_achieved": round(algo_rd / per_launch_s / 1e9, 1),
                     "read_frac": round(algo_rd / per_launch_s / 1e9 / HBM_PEAK_GBS, 4),
                     "kernel": kernel, "traffic_source": traffic_src,
                     "timing": "HIP events around each whole step on the engine stream "
                               "(one tlsgpu_open_batch: with the stated hints the fused queue "
                               "kernel alone, its prologue doing the bounds check, statuses and "
                               "per-record constants; else bounds + prep passes + main kernels)",
                     **comp},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if rec_len:
            line["cpu_baseline"] = cpu_baseline(kind_name, rec_len, op)
        else:  # mixed lengths: the first 16 Ki records of the workload's own Zipf mix
            line["cpu_baseline"] = cpu_baseline(kind_name, lengths[:16384], op)
    if rank == 0:
        print(json.dumps(line), flush=True)
    ev0.close()
    ev1.close()
    wl.free()
    cp.close()
    eng.close()


def settle(step, sync, ms: float) -> dict:
    """Untimed back-to-back steps for >= `ms` of wall time (synchronising every
    8 steps to read the clock): the GPU's power governor leaves the clock dip
    of a fresh sustained load before the warm-up and the timed region."""
    if ms <= 0:
        return {"ms": 0.0, "steps": 0}
    n, t0 = 0, time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            step()
        n += 8
        sync()
    return {"ms": round((time.perf_counter() - t0) * 1e3, 1), "steps": n}


def choose_split(split: str | None, world: int, devices: str, gpus: int = 1) -> str:
    """The multi-GPU split a run measures: the C ABI's group split for N > 1 GPUs
    — asked for by --gpus N (with or without a launcher), by N > 1 ranks or by
    an explicit device list — one engine per rank otherwise."""
    if split:
        return split
    return "group" if world > 1 or gpus > 1 or devices else "ranks"


def group_devices(devices: str, gpus: int, world: int) -> list[int]:
    """Member devices of the group: the list given, else 0..N-1 with N the
    larger of --gpus and the launcher's world size."""
    if devices:
        out = [int(x) for x in devices.split(",") if x.strip() != ""]
        if not out or min(out) < 0:
            raise SystemExit(f"bad --devices {devices!r}")
        return out
    return list(range(max(gpus, world, 1)))


def check_devices(devices: list[int], visible: int, explicit: bool) -> None:
    """A run that asks for N GPUs measures N distinct GPUs or fails: exit
    non-zero when a member device is not visible.  An explicit --devices list
    may repeat an id on purpose (the '0,0' one-GPU rehearsal), never name an
    invisible one."""
    if visible <= 0:
        raise SystemExit("no GPU visible")
    if max(devices) >= visible:
        raise SystemExit(f"{len(devices)} GPUs asked for (devices {devices}) but only {visible} "
                         "visible: refusing to measure fewer")
    if not explicit and len(set(devices)) != len(devices):
        raise SystemExit(f"duplicate devices {devices}")


def group_mode(args, world, rank):
    """Config E through the C ABI's own batch split (include/tlsgpu.h
    tlsgpu_group_*, talos_amd/csrc/group.cpp): ONE process creates a group of
    N member engines (one per device), member k builds shard k of config E's
    batch in its own HBM (talos_amd.workload, global record indices, as
    tests/golden/batch_digests.json E_shard<k> pins), the session table is
    replicated on every member (tlsgpu_group_sessions_install), and each step
    is one tlsgpu_group_open_batch — every member's open launched on its own
    stream from the caller's thread — joined by tlsgpu_group_sync.  Under
    torch.distributed.run (N ranks) rank 0 drives the whole group and the
    other ranks only join the gloo barrier (they never touch a GPU)."""
    import talos_amd as ta
    from talos_amd.dist import ControlPlane, shard_by_bytes
    from talos_amd.workload import Workload, session_plan

    cp = ControlPlane(world)
    if rank != 0:
        cp.barrier()
        cp.close()
        return
    ta.load_library()
    devices = group_devices(args.devices, args.gpus, world)
    check_devices(devices, ta.device_count(), bool(args.devices))
    n = len(devices)
    cfg = "E" if args.config in ("B", "E") else args.config
    if cfg != "E":
        raise SystemExit("--split group runs config E (configs[4]) only")
    kind_name, per_gpu, sessions, rec_len, seed, op = CONFIGS[cfg]
    if args.records:
        per_gpu = args.records
    kind = ta.AEAD_NAMES[kind_name]
    shards = max(E_GPUS, n)
    glob = np.full(shards * per_gpu, rec_len, dtype=np.int64)
    g = ta.Group(devices)
    members = [ta.Engine.member(g, k) for k in range(n)]
    wls = []
    for k in range(n):
        lo, hi = shard_by_bytes(glob, shards, k)
        wls.append(Workload(members[k], kind, shards * per_gpu, shards * sessions, seed,
                            record_len=rec_len, tamper_every=1024, shard=(lo, hi)))
    # the group's session table, replicated on every member: every session the
    # members' shards use, at its global id
    n_sess = max(wl.s0 + wl.S for wl in wls)
    params = session_plan(kind, shards * per_gpu, shards * sessions, seed)[0][:n_sess]
    gs = ta.GroupSessionTable(g, n_sess)
    gs.install(0, params)
    shard_arr = np.zeros(n, dtype=ta.SHARD_DTYPE)
    d_descs = []
    for k, wl in enumerate(wls):
        opn = wl.d_open.download().view(ta.RECORD_DTYPE).copy()
        opn["session"] += np.uint32(wl.s0)     # workload-local ids -> global ids
        d = ta.DeviceBuffer(members[k], opn.nbytes)
        d.upload(opn.view(np.uint8))
        d_descs.append(d)
        shard_arr[k] = (d.ptr, wl.n, 0, wl.d_body.ptr, wl.d_body.nbytes, wl.d_out.ptr,
                        wl.d_out.nbytes, wl.d_status.ptr)
        hints = 0 if args.no_hints else ta.batch_hints(
            wl.lengths + ta.EXPLICIT_NONCE_LEN[kind] + ta.TAG_LEN, wl.session, seal=False)
        ta._check(g.lib.tlsgpu_sessions_hint(g.lib.tlsgpu_group_sessions_member(gs.handle, k),
                                             hints), "tlsgpu_sessions_hint")
    gs.batch(shard_arr, seal=False)     # verified first, then warmed (as the device mode)
    g.sync()
    for wl in wls:
        wl.verify_open()
    evs = [(ta.Event(m), ta.Event(m)) for m in members]
    settled = settle(lambda: gs.batch(shard_arr, seal=False), g.sync, args.settle_ms)
    for _ in range(max(1, args.warmup)):
        gs.batch(shard_arr, seal=False)
    g.sync()
    t0 = time.perf_counter()
    for e0, _ in evs:
        e0.record()
    for _ in range(args.steps):
        gs.batch(shard_arr, seal=False)
    for _, e1 in evs:
        e1.record()
    g.sync()
    wall_s = time.perf_counter() - t0
    dev_ms = [e0.elapsed_ms(e1) for e0, e1 in evs]
    for wl in wls:
        wl.verify_open()
    total_len = sum(int(wl.lengths.sum()) for wl in wls)
    # the same timing method as N = 1: HIP events around the K steps on each
    # member's stream; the slowest member sets the step time (max over GPUs,
    # as max over ranks); wall clock as a second field
    slowest_s = max(dev_ms) / 1e3
    value = total_len * args.steps / slowest_s / GIB
    per_launch_s = slowest_s / args.steps
    algo = sum(algo_bytes_per_record(kind_name, int(l), op) for l in wls[0].lengths.tolist())
    algo_rd = sum(algo_bytes_per_record(kind_name, int(l), op, True)
                  for l in wls[0].lengths.tolist())
    kernel = main_kernel(kind_name, op, False, False, wls[0].n)
    traffic, traffic_src = load_traffic("B", kernel)
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": n,
        "steps": args.steps, "warmup": args.warmup, "settle": settled,
        "ms_per_step": round(slowest_s * 1e3 / args.steps, 4),
        "wall_ms_per_step": round(wall_s * 1e3 / args.steps, 4),
        "wall_value": round(total_len * args.steps / wall_s / GIB, 3),
        "member_device_ms_per_step": [round(x / args.steps, 4) for x in dev_ms],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (counter-SplitMix64 plaintexts sealed on device; 1/1024 tampered)",
        "config": {"workload": f"config E: {kind_name} TLS 1.2 record open, 16 KiB records, "
                               f"{per_gpu} records/GPU, device-resident; shards 0..{n - 1} of "
                               f"one {shards * per_gpu}-record batch (seed {seed:#x}, "
                               f"{shards * sessions} sessions)",
                   "records_per_gpu": per_gpu, "sessions_per_gpu": sessions,
                   "devices": devices, "split": "tlsgpu_group_open_batch (C ABI, group.cpp): "
                   "one process, one member engine per device, replicated session table",
                   "payload_bytes_per_gpu": int(wls[0].lengths.sum()),
                   "parallelism": f"batch split x{n} (tlsgpu_group)"},
        "roofline": {"bound": "hbm", "achieved": round(algo / per_launch_s / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(algo / per_launch_s / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "algorithmic_bytes_per_launch": algo,
                     "read_achieved": round(algo_rd / per_launch_s / 1e9, 1),
                     "read_frac": round(algo_rd / per_launch_s / 1e9 / HBM_PEAK_GBS, 4),
                     "kernel": kernel, "traffic_source": traffic_src,
                     "timing": "HIP events around the K steps on every member's stream; "
                               "value and ms_per_step from the slowest member (as N = 1 from "
                               "its one stream); wall_value: wall clock around the K group "
                               "calls + tlsgpu_group_sync"},
    }
    if n == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(kind_name, rec_len, op)
    print(json.dumps(line), flush=True)
    for e0, e1 in evs:
        e0.close()
        e1.close()
    for d in d_descs:
        d.free()
    for wl in wls:
        wl.free()
    gs.close()
    g.close()
    cp.barrier()
    cp.close()


def copy_mode(args, eng):
    """Achievable HBM bandwidth on this box: hipMemcpyAsync device-to-device of
    1 GiB (read 1 GiB + write 1 GiB per step), HIP events on the engine stream."""
    import talos_amd as ta
    nbytes = 1 << 30
    a, b = ta.DeviceBuffer(eng, nbytes), ta.DeviceBuffer(eng, nbytes)
    a.fill(0x5A)
    ev0, ev1 = ta.Event(eng), ta.Event(eng)
    for _ in range(max(1, args.warmup)):
        b.copy_from(a)
    eng.sync()
    ev0.record()
    for _ in range(args.steps):
        b.copy_from(a)
    ev1.record()
    ms = ev0.elapsed_ms(ev1) / args.steps
    print(json.dumps({"metric": "device-to-device copy bandwidth (hipMemcpyAsync, 1 GiB)",
                      "value": round(2 * nbytes / (ms / 1e3) / 1e9, 1), "unit": "GB/s",
                      "note": "read + written bytes / time", "ms_per_copy": round(ms, 4),
                      "frac_of_8TBs": round(2 * nbytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                      "steps": args.steps}), flush=True)
    for x in (a, b):
        x.free()
    eng.close()


def host_mode(args, eng, wl, kind_name, total_len):
    """PCIe-inclusive rate (north_star: the path starts and ends in host memory):
    pinned host fragments in, pinned host plaintext out, through the C-ABI
    tlsgpu_open_host (chunked multi-stream H2D / kernel / D2H pipeline)."""
    import talos_amd as ta
    from talos_amd.pipeline import HostPipeline
    if args.host_streams or args.host_chunk_mib:
        ta.host_pipeline(eng, args.host_streams, args.host_chunk_mib << 20)
    pipe = HostPipeline(wl)
    for _ in range(max(1, args.warmup)):
        pipe.run()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.run()
    dt = time.perf_counter() - t0
    # every status exact; sampled plaintexts equal the originals, tampered zeroed
    st = pipe.status()
    want = np.where(wl.tampered, -1, wl.lengths).astype(np.int32)
    assert np.array_equal(st, want), int((st != want).sum())
    rng = np.random.default_rng(1)
    for i in list(rng.choice(wl.n, 32, replace=False)) + list(np.nonzero(wl.tampered)[0][:4]):
        got = pipe.host_plaintext(int(i))
        exp = (bytes(int(wl.lengths[i])) if wl.tampered[i] else
               wl.d_pt.download(int(wl.lengths[i]), int(wl.pt_off[i])).tobytes())
        assert got == exp, i
    print(json.dumps({"metric": f"GiB/s host-resident {kind_name} TLS record open "
                                "(tlsgpu_open_host: pinned H2D + kernels + D2H, pipelined)",
                      "value": round(total_len * args.steps / dt / GIB, 3), "unit": "GiB/s",
                      "steps": args.steps, "records": wl.n,
                      "h2d_bytes_per_step": wl.body_bytes, "d2h_bytes_per_step": wl.pt_bytes,
                      "ms_per_step": round(dt * 1e3 / args.steps, 3),
                      "compute_streams": args.host_streams or 2, "chunk_mib": args.host_chunk_mib or 32,
                      "timing": "wall clock around each synchronous tlsgpu_open_host call"}),
          flush=True)
    pipe.close()
    wl.free()
    eng.close()


def pcie_mode(args, eng):
    """Raw pinned-host <-> HBM copy rates of this box (the ceiling of --mode host):
    1 GiB H2D alone, D2H alone, and both at once on two streams."""
    import ctypes as C
    import talos_amd as ta
    lib = eng.lib
    nbytes = 1 << 30
    h1, h2 = C.c_void_p(), C.c_void_p()
    ta._check(lib.tlsgpu_host_alloc(eng.handle, nbytes, C.byref(h1)), "host_alloc")
    ta._check(lib.tlsgpu_host_alloc(eng.handle, nbytes, C.byref(h2)), "host_alloc")
    d1, d2 = ta.DeviceBuffer(eng, nbytes), ta.DeviceBuffer(eng, nbytes)
    s1, s2 = eng.new_stream(), eng.new_stream()
    C.memset(h1, 0x5A, nbytes)
    res = {}
    for name, jobs in (("h2d", [(d1.ptr, h1.value, s1)]), ("d2h", [(h2.value, d2.ptr, s2)]),
                       ("both", [(d1.ptr, h1.value, s1), (h2.value, d2.ptr, s2)])):
        for rep in range(2):
            t0 = time.perf_counter()
            for dst, src, s in jobs:
                ta._check(lib.tlsgpu_memcpy(eng.handle, dst, src, nbytes, s), "memcpy")
            for _, _, s in jobs:
                eng.sync_stream(s)
            dt = time.perf_counter() - t0
        res[name + "_GBps"] = round(len(jobs) * nbytes / dt / 1e9, 2)
    print(json.dumps({"metric": "pinned host <-> HBM copy rate (hipMemcpyAsync, 1 GiB)", **res}),
          flush=True)
    lib.tlsgpu_host_free(eng.handle, h1)
    lib.tlsgpu_host_free(eng.handle, h2)
    d1.free()
    d2.free()
    eng.close()


def wire_mode(args, eng, wl, kind_name, total_len):
    """Raw wire streams (one per session = connection direction, its records back
    to back as 5-B header + fragment) through tlsgpu_open_wire: device framing
    (ssl3_get_record's header walk) + in-place open + alert mapping.  Fragments
    sit at wire offsets, i.e. mostly not 16-B aligned, as on a real socket
    buffer.  The wire is restored from a pristine copy before every step (in-place
    open overwrites it); only the open_wire calls are timed (HIP events)."""
    import talos_amd as ta
    eiv = ta.EXPLICIT_NONCE_LEN[wl.kind]
    body = wl.d_body.download()
    frag = (wl.lengths + eiv + ta.TAG_LEN).astype(np.int64)
    parts, descs, frag_pos = [], [], np.zeros(wl.n, dtype=np.int64)
    pos = 0
    for s in range(wl.S):
        idx = np.nonzero(wl.session == s)[0]
        if len(idx) == 0:
            continue
        start = pos
        for i in idx:
            fl = int(frag[i])
            parts.append(np.frombuffer(bytes([23, 3, 3, fl >> 8, fl & 0xFF]), dtype=np.uint8))
            o = int(wl.body_off[i])
            parts.append(body[o:o + fl])
            frag_pos[i] = pos + 5
            pos += 5 + fl
        descs.append((start, pos - start, s, int(wl.seq[idx[0]]), 0x0303, 0, 0))
    wire = np.concatenate(parts)
    del parts, body
    ns = len(descs)
    d_streams = ta.DeviceBuffer(eng, ns * ta.WIRE_STREAM_DTYPE.itemsize)
    d_streams.upload(np.array(descs, dtype=ta.WIRE_STREAM_DTYPE).view(np.uint8))
    d_wire0 = ta.DeviceBuffer(eng, len(wire) + 64)
    d_wire0.upload(np.concatenate([wire, np.zeros(64, np.uint8)]))
    d_wire = ta.DeviceBuffer(eng, len(wire) + 64)
    d_recs = ta.DeviceBuffer(eng, 32 * wl.n)
    d_status = ta.DeviceBuffer(eng, 4 * wl.n)
    d_results = ta.DeviceBuffer(eng, ta.WIRE_RESULT_DTYPE.itemsize * ns)
    d_total = ta.DeviceBuffer(eng, 4)
    evs = [ta.Event(eng) for _ in range(2)]

    def step():
        d_wire.copy_from(d_wire0)
        evs[0].record()
        ta.open_wire(wl.table, d_streams.ptr, ns, d_wire.ptr, wl.n, d_recs.ptr, d_status.ptr,
                     d_results.ptr, d_total.ptr)
        evs[1].record()
        eng.sync()
        return evs[0].elapsed_ms(evs[1])

    for _ in range(max(1, args.warmup)):
        step()
    ms = [step() for _ in range(args.steps)]
    # verify: every stream fully framed and delivered, statuses exact, sampled plaintexts
    res = d_results.download().view(ta.WIRE_RESULT_DTYPE)
    assert int(d_total.download().view(np.uint32)[0]) == wl.n
    assert (res["alert"] == 0).all() and int(res["delivered"].sum()) == wl.n
    assert (res["consumed"].astype(np.int64) == np.array([d[1] for d in descs])).all()
    recs = d_recs.download().view(ta.RECORD_DTYPE)
    st = d_status.download().view(np.int32)
    by_off = {int(r["in_off"]): k for k, r in enumerate(recs)}
    rng = np.random.default_rng(wl.seed)
    for i in rng.choice(wl.n, size=min(32, wl.n), replace=False):
        k = by_off[int(frag_pos[i])]
        assert st[k] == wl.lengths[i], (i, st[k])
        ln, o = int(wl.lengths[i]), int(frag_pos[i]) + eiv
        got = d_wire.download(ln, o)
        assert np.array_equal(got, wl.d_pt.download(ln, int(wl.pt_off[i]))), i
    avg = sum(ms) / len(ms)
    mis = int(((frag_pos + eiv) % 16 != 0).sum())
    print(json.dumps({
        "metric": f"GiB/s device-resident {kind_name} TLS wire-stream open (tlsgpu_open_wire: "
                  "framing + in-place open + alerts)",
        "value": round(total_len / (avg / 1e3) / GIB, 3), "unit": "GiB/s", "steps": args.steps,
        "ms_per_step": round(avg, 4), "records": wl.n, "streams": ns,
        "payload_bytes": total_len, "wire_bytes": int(len(wire)),
        "records_not_16B_aligned": mis, "gcm_impl": ta.get_gcm_impl(),
        "timing": "HIP events around each tlsgpu_open_wire call; wire restored between steps"}),
        flush=True)
    for b in (d_streams, d_wire0, d_wire, d_recs, d_status, d_results, d_total):
        b.free()
    wl.free()
    eng.close()


if __name__ == "__main__":
    main()
