"""Benchmark: scanned GB/s per GPU of the MI355X Aho-Corasick atom scanner.

Metric (BASELINE.json): "scanned GB/s per GPU (4 GiB buffer, 10k atoms) +
bit-exact match-set vs CPU".  Workload = config C: the 10k mixed hex/ascii/
wildcard rule set (tests/golden/tables/C.npz, compiled by stock libyara), 4 GiB
of the canonical xorshift64 input per GPU, resident in HBM before timing.

A step = one pass of the hot path over the batch: the scan kernel over the
whole shard, candidate compaction into one ascending position array, and for
N > 1 the RCCL gather of every rank's candidate list to rank 0 (config D:
one logical 4N GiB buffer, rank r owns bytes [4r, 4r+4) GiB and holds them
plus the rule set's verify halos, yara_amd/dist.py; weak scaling).  The
line's "verified_step" times the verification-complete step separately: the
same plus on-device pre-verification per rank and, for N > 1, the gather of
the pre-verified {offset, pool index} records.  "other_rule_sets" (N = 1):
the scan kernel of other rule-set shapes, and for the dense 1-byte-key sets
(rx, short, fuzz0, fuzz3) their verified-only step (verified_step_ms: scan,
result and pre-verification on the host's clock).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no launcher around it (WORLD_SIZE unset) bench.py starts
the N rank processes itself, before anything touches the GPU, with torchrun's
environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, ...), and
exits with the worst rank's code; --launch-only prints those environments.

Clocks: from idle the scan kernel's first launches take up to 1.2 ms and
settle at ~0.86 ms after ~25 ms of kernel time.  Every rank, for every N,
first scans back to back for --clock-warmup-s seconds (default 0.4 s, ~450
scans) before any measured leg, so the headline of N = 1 and of N > 1 is taken
on the same settled clock; W warm-up steps follow as usual.

Rank 0 prints one JSON line.  value = total bytes scanned by all ranks per
second (decimal GB/s).  roofline = the scan kernel's algorithmic HBM bytes
(1 B per input byte) per launch / its HIP-event duration, vs
the 8.0 TB/s HBM3E peak.  cpu_baseline = the stock reference libyara
(oracle/_ref) on the host, one YR_SCANNER per thread, a bounded sample, at the
faster of: every CPU the process may run on, and the CPUs its cgroup grants;
the 1-thread stock yr_rules_scan_mem beside it.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

GiB = 1 << 30
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--rules", default="C", help="rule set (tests/golden/tables/<name>.npz)")
    ap.add_argument("--gib-per-gpu", type=float, default=4.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-sample-mib", type=int, default=3072)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--no-other", action="store_true",
                    help="skip the other rule sets' kernel timings (B, E, rx, short, fuzz0, fuzz3)")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL) or gloo (rehearsal)")
    ap.add_argument("--dist", action="store_true",
                    help="run the N > 1 code path (process group, per-rank attribution, "
                         "gathers) even at world size 1")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the multi-threaded CPU baselines (0: every CPU this "
                         "process may run on)")
    ap.add_argument("--clock-warmup-s", type=float, default=0.4,
                    help="back-to-back scans before the measured legs, on every rank")
    ap.add_argument("--launch-only", action="store_true",
                    help="with --gpus N > 1 and no launcher: print the N rank environments "
                         "this process would start, as one JSON line, and exit")
    ap.add_argument("--rank-probe", action="store_true",
                    help="(test hook) each rank prints its rank environment as JSON and exits "
                         "before importing torch; --rank-probe-fail R makes rank R exit 3")
    ap.add_argument("--rank-probe-fail", type=int, default=-1, help=argparse.SUPPRESS)
    return ap.parse_args()


RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
            "MASTER_ADDR", "MASTER_PORT")


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n: int, port: int):
    """The environments of the N rank processes of one node, as torchrun sets
    them (one process per GPU, rendezvous on 127.0.0.1)."""
    return [{"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
             "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
             "MASTER_PORT": str(port)} for r in range(n)]


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) run without a launcher: start the N ranks
    here, as fresh child processes of this script with torchrun's environment,
    BEFORE this process touches the GPU (it never does: torch is not even
    imported), wait for all of them and return the worst exit code.  Rank 0's
    stdout carries the JSON line.  A rank that fails ends the others (their
    exact PIDs), so no rank is left waiting in a collective; a rank that cannot
    be started is a non-zero exit -- never a 1-GPU line for --gpus N."""
    import signal
    import subprocess
    port = _free_port()
    envs = rank_envs(args.gpus, port)
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    if args.launch_only:
        print(json.dumps({"launcher": "bench.py", "cmd": cmd, "ranks": envs}), flush=True)
        return 0
    procs = []
    try:
        for e in envs:
            env = dict(os.environ)
            env.update(e)
            procs.append(subprocess.Popen(cmd, env=env))
    except OSError as ex:
        print("bench.py: could not start rank %d: %s" % (len(procs), ex), file=sys.stderr)
        for p in procs:
            p.send_signal(signal.SIGTERM)
        for p in procs:
            p.wait()
        return 1
    # a launcher that stops us (timeout, Ctrl-C) stops the ranks too: no rank
    # is left holding a GPU
    def forward(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        sys.exit(128 + signum)
    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    worst = 0
    live = list(procs)
    term_at = None
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and term_at is None:
                worst = rc if rc > 0 else 128 - rc
                term_at = time.monotonic()
                for q in live:               # the rest would wait in a collective
                    q.send_signal(signal.SIGTERM)
        if live and term_at is not None and time.monotonic() - term_at > 30:
            for q in live:
                q.kill()
            term_at = float("inf")
        time.sleep(0.05)
    return worst


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def cpu_info():
    """What the host offers this process: nproc, the CPUs it may run on, and
    the cgroup CPU quota if one is set (a GPU box shares its host)."""
    info = {"model": cpu_model(), "nproc": os.cpu_count() or 0}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = info["nproc"]
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        info["cgroup_cpu_max"] = " ".join(q)
        if q[0] != "max":
            info["cgroup_cpus"] = round(int(q[0]) / int(q[1]), 2)
    except (OSError, ValueError, IndexError):
        pass
    return info


def _stock_rules(rules: str):
    ref_so = os.path.join(REPO, "oracle", "_ref", "libyara_ref.so")
    if not os.path.exists(ref_so):
        return None, None
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen_rules
    return ref_so, gen_rules.gen(rules).encode()


def cpu_baseline(rules: str, data, seed: int):
    """Stock reference libyara yr_rules_scan_mem on the host (kind "reference"),
    or the in-repo restatement of scanner.c:45-176 (kind "port") if the
    reference build did not travel.  1 thread, a bounded prefix of the input."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import oracle
    n = data.size
    ref_so, src = _stock_rules(rules)
    if ref_so is not None:
        L = ctypes.CDLL(ref_so)
        L.yr_initialize()
        comp = ctypes.c_void_p()
        assert L.yr_compiler_create(ctypes.byref(comp)) == 0
        L.yr_compiler_add_string.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
        assert L.yr_compiler_add_string(comp, src, None) == 0
        rules_h = ctypes.c_void_p()
        L.yr_compiler_get_rules.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
        assert L.yr_compiler_get_rules(comp, ctypes.byref(rules_h)) == 0
        CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                              ctypes.c_void_p)
        cb = CB(lambda ctx, msg, md, ud: 0)   # CALLBACK_CONTINUE
        L.yr_rules_scan_mem.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_int, CB, ctypes.c_void_p, ctypes.c_int]
        t0 = time.perf_counter()
        rc = L.yr_rules_scan_mem(rules_h, data.ctypes.data, n, 0, cb, None, 0)
        dt = time.perf_counter() - t0
        L.yr_compiler_destroy(comp)
        L.yr_rules_destroy(rules_h)
        L.yr_finalize()                           # paired with yr_initialize above
        assert rc == 0, rc
        kind, what = "reference", "stock libyara 4.2.1 yr_rules_scan_mem (oracle/_ref)"
    else:
        from conftest import ref_tables   # noqa
        tab = ref_tables(rules)
        t0 = time.perf_counter()
        oracle.count_parallel(tab, data, 1)
        dt = time.perf_counter() - t0
        kind, what = "port", "in-repo restatement of scanner.c:45-176 (oracle/ac_oracle.c)"
    return {"value": round(n / dt / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": kind,
            "sample": "%s, rule set %s, first %d MiB of the xorshift64 seed-%d input, 1 thread, "
                      "%.1f s, %s (nproc %d)" % (what, rules, n >> 20, seed, dt, cpu_model(),
                                                 os.cpu_count() or 0)}


def cpu_stock_threads(rules: str, data, seed: int, threads: int, min_s: float = 3.0):
    """SURVEY.md §8d's multi-threaded CPU comparator on STOCK libyara:
    `threads` threads, each with its own YR_SCANNER (yr_scanner_create, as
    cli/yara.c:1564-1608 gives each scanning thread one) scanning its own
    contiguous slice of the sample with a 4-byte warm-up, passes repeated for
    at least `min_s` seconds (oracle/refmt.c, built against oracle/_ref)."""
    ref_so, src = _stock_rules(rules)
    mt_so = os.path.join(REPO, "oracle", "_ref", "librefmt.so")
    if ref_so is None or not os.path.exists(mt_so):
        return None
    L = ctypes.CDLL(mt_so)
    L.refmt_scan.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                             ctypes.c_double, ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double)]
    gbps, passes, secs = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_double()
    rc = L.refmt_scan(src, data.ctypes.data, data.size, threads, min_s, ctypes.byref(gbps),
                      ctypes.byref(passes), ctypes.byref(secs))
    if rc != 0:
        return {"error": "refmt_scan returned %d" % rc}
    info = cpu_info()
    return {"value": round(gbps.value, 3), "unit": "GB/s", "cores": threads, "kind": "reference",
            "sample": "stock libyara 4.2.1 (oracle/_ref), %d threads x one YR_SCANNER each over "
                      "contiguous slices (4-byte warm-up) of the first %d MiB of the xorshift64 "
                      "seed-%d input, rule set %s, %d pass(es) in %.1f s (oracle/refmt.c)"
                      % (threads, data.size >> 20, seed, rules, passes.value, secs.value),
            "host": info}


def cpu_parallel(rules: str, data, threads: int, min_s: float = 2.0):
    """the in-repo restatement of scanner.c:45-176, one walker
    per contiguous slice with a 4-byte warm-up, `threads` threads, repeated for
    at least `min_s` seconds (reported beside cpu_baseline)."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import oracle
    from conftest import ref_tables   # noqa
    tab = ref_tables(rules)
    passes = 0
    t0 = time.perf_counter()
    while True:
        oracle.count_parallel(tab, data, threads)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= min_s:
            break
    return {"value": round(data.size * passes / dt / 1e9, 3), "unit": "GB/s", "cores": threads,
            "kind": "port", "sample": "oracle/ac_oracle.c slice walkers, rule set %s, first %d MiB, "
            "%d pass(es) in %.1f s" % (rules, data.size >> 20, passes, dt)}


def load_traffic(kernel_bytes):
    """HBM bytes per scan-kernel launch from the committed PMC pass: a
    separate `rocprofv3 --pmc FETCH_SIZE` run of this bench (tools/
    profile_round.sh -> tools/pmc_summary.py -> profiles/pmc_traffic.json;
    counters cannot be collected inside the timed run).  Returns (bytes,
    source) -- the source names the file and the round/commit it was measured
    at, so a stale profile is visible as such -- or (None, reason)."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, "no PMC pass committed (profiles/pmc_traffic.json)"
    try:
        d = json.load(open(p))
        if int(d.get("input_bytes", -1)) == kernel_bytes:
            return (int(d["hbm_bytes_per_launch"]),
                    "profiles/pmc_traffic.json: rocprofv3 --pmc FETCH_SIZE (x2 gfx950 "
                    "correction), %s" % d.get("measured", "round r01"))
    except Exception:
        pass
    return None, "profiles/pmc_traffic.json is for another input size"


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher (torchrun) around us: start the N ranks ourselves
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.rank_probe:
        print(json.dumps({k: os.environ.get(k) for k in RANK_ENV}), flush=True)
        if args.rank_probe_fail >= 0 and rank != args.rank_probe_fail:
            time.sleep(120)                  # stands for a rank waiting in a collective
        sys.exit(3 if rank == args.rank_probe_fail else 0)

    sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch
    import torch.distributed as dist

    import yara_amd
    from yara_amd._hip import memcpy
    # the N > 1 code path: a process group, per-rank attribution, the gathers
    # (--dist: also at world size 1, e.g. RCCL on one GPU)
    use_dist = world > 1 or args.dist
    if use_dist and world == 1:
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29533"), ("RANK", "0"),
                     ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible")
    if use_dist and args.backend == "nccl" and world > ndev:
        # two RCCL ranks cannot share one device; rehearse with --backend gloo
        raise SystemExit("bench.py: --gpus %d with backend nccl but only %d GPU(s) visible"
                         % (world, ndev))
    dev = torch.device("cuda", local % ndev)   # % ndev: gloo rehearsals on fewer GPUs
    torch.cuda.set_device(dev)
    if use_dist:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    from yara_amd import dist as ydist
    tables = yara_amd.Tables.from_npz(os.path.join(REPO, "tests", "golden", "tables",
                                                   "%s.npz" % args.rules), device=dev.index,
                                      strings=True)
    shard = int(args.gib_per_gpu * GiB)
    total = shard * world                           # one logical block, sharded
    begin, end = ydist.shard_bounds(total, world, rank)
    begins_all = [ydist.shard_bounds(total, world, r)[0] for r in range(world)]
    # the rank's window of the block: its shard plus the tables' verify halos
    # (yr_amd_tables_info), so on-device pre-verification of its own candidates
    # is exactly the whole block's (dist.py); N = 1: the whole block
    halo_before, halo_after = ydist.tables_halos(tables)
    lo, hi = ydist.shard_window(total, begin, end, halo_before, halo_after)
    buf = torch.empty(hi - lo + 16, dtype=torch.uint8, device=dev)
    yara_amd.fill_xorshift64(buf.data_ptr(), hi - lo, args.seed, lo)
    torch.cuda.synchronize()

    stream = torch.cuda.Stream(device=dev)
    # DEPTH scanners on ONE stream, used in turn: the scans of steps k+1 ..
    # k+DEPTH-1 are queued before the host collects step k's result
    # (yr_amd_scan_device_result waits on the scan's own event), so the GPU does
    # not idle while the host -- or, with N > 1, the RCCL gather -- turns a
    # result around; the kernels still run one after another, so the
    # per-kernel timing is unaffected
    depth = 3
    scanners = [yara_amd.Scanner(tables, stream=stream.cuda_stream) for _ in range(depth)]
    scanner = scanners[0]

    def launch(k):
        scanners[k % depth].scan_window(buf.data_ptr(), lo, hi, total, begin, end)

    gather_s = [0.0]   # wall time of this rank's gathers (N > 1), timed steps only

    def finish(k, timed_kernel=False):
        sc = scanners[k % depth]
        ptr, cnt, _ = sc.device_result()            # ascending block positions in HBM
        kms = sc.kernel_ms() if timed_kernel else None
        if not use_dist:
            return (ptr, cnt), kms
        t_g = time.perf_counter()
        pos = torch.empty(max(cnt, 1), dtype=torch.int64, device=dev)
        memcpy(pos.data_ptr(), ptr, cnt * 8, 3)
        # RCCL: counts + padded gather of 32-bit offsets from each shard's begin
        pos = ydist.gather_positions(pos[:cnt], begins=begins_all, end=total)
        if timed_kernel:
            gather_s[0] += time.perf_counter() - t_g
        return pos, kms

    def run(steps, timed_kernel=False):
        out, kms = None, []
        for k in range(steps):
            launch(k)
            if k >= depth - 1:
                out, t = finish(k - depth + 1, timed_kernel)
                kms.append(t)
        for k in range(max(0, steps - depth + 1), steps):
            out, t = finish(k, timed_kernel)
            kms.append(t)
        return out, kms

    # Clock warm-up, the same on every rank for every N: back-to-back scans of
    # the rank's own window for a fixed wall time (from idle the scan kernel's
    # first launches take up to 1.2 ms and settle at ~0.86 ms over ~25 ms of
    # work, profiles/r02_baseline_kernel_stats.csv -- W = 5 warm-up steps alone
    # do not cover that).
    t_w = time.perf_counter()
    n_clock = 0
    while time.perf_counter() - t_w < args.clock_warmup_s:
        launch(n_clock)
        if n_clock >= depth - 1:
            scanners[(n_clock - depth + 1) % depth].device_result()
        n_clock += 1
    for k in range(max(0, n_clock - depth + 1), n_clock):
        scanners[k % depth].device_result()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    # Order of the legs: the secondary measurements first (the other rule sets'
    # kernel times, the verification-complete step), the headline last.
    # the same input under the other rule sets of SURVEY.md §8d (kernel time only,
    # not the bench value): B = 1,000 4-byte hex atoms, E = 2,000 nocase/masked;
    # and the shapes with 1-byte keys, whose candidates are dense:
    # rx = regexps, short = short literals, fuzz0 / fuzz3 = generated rule sets
    other = None
    if rank == 0 and world == 1 and not args.no_other and args.rules == "C":
        other = {}
        for name in ("B", "E", "rx", "short", "fuzz0", "fuzz3"):
            t_o = yara_amd.Tables.from_npz(os.path.join(REPO, "tests", "golden", "tables",
                                                        "%s.npz" % name), device=dev.index)
            s_o = yara_amd.Scanner(t_o, stream=stream.cuda_stream)
            for _ in range(20):
                s_o.scan_device(buf.data_ptr(), total)
                s_o.device_result()
            s_o.set_timing(True)
            ks = []
            for _ in range(20):
                s_o.scan_device(buf.data_ptr(), total)
                _, c_o, _ = s_o.device_result()
                ks.append(s_o.kernel_ms())
            k_o = sum(ks) / len(ks)
            other[name] = {"kernel_ms": round(k_o, 4),
                           "GB/s": round(shard / (k_o * 1e-3) / 1e9, 1),
                           "frac": round(shard / (k_o * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "candidates": int(c_o)}
            del s_o, t_o
            if name in ("rx", "short", "fuzz0", "fuzz3"):
                # the verified path of the dense sets (tools/ruleset_rates.py's
                # verified-only leg): tables with their string records, scan +
                # result + on-device pre-verification per step, host clock,
                # median of 20 steps after 0.5 s of them (clock ramp)
                t_v = yara_amd.Tables.from_npz(os.path.join(REPO, "tests", "golden", "tables",
                                                            "%s.npz" % name), device=dev.index, strings=True)
                s_v = yara_amd.Scanner(t_v, stream=stream.cuda_stream)
                s_v.set_verified_only(True)

                def v_step():
                    s_v.scan_device(buf.data_ptr(), total)
                    s_v.device_result()
                    return s_v.verify_device(0)[1]
                t_w = time.perf_counter()
                while time.perf_counter() - t_w < 0.5:
                    v_step()
                ws = []
                for _ in range(20):
                    torch.cuda.synchronize()
                    t_s = time.perf_counter()
                    n_v = v_step()
                    ws.append((time.perf_counter() - t_s) * 1e3)
                ws.sort()
                w_med = (ws[9] + ws[10]) / 2
                other[name]["verified_step_ms"] = round(w_med, 4)
                other[name]["verified_frac"] = round(shard / (w_med * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                other[name]["verified_records"] = int(n_v)
                del s_v, t_v

    # The verification-complete step, timed separately over the same number of
    # steps (not the bench value): scan + compaction + on-device
    # pre-verification of the rank's candidates (yr_amd_verify_device) and, for
    # N > 1, the RCCL gather of the {offset, pool index} records to rank 0 --
    # i.e. everything the host's yr_scan_verify_match still has to see.
    def verified_step():
        scanner.scan_window(buf.data_ptr(), lo, hi, total, begin, end)
        scanner.device_result()
        ptr, n_rec = scanner.verify_device(0)
        if use_dist:
            return ydist.gather_rows(ydist.records_to_rows(ptr, n_rec, dev))
        return n_rec
    for _ in range(max(args.warmup, 3)):
        verified_step()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        v_out = verified_step()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    v_elapsed = time.perf_counter() - t0
    if use_dist:
        t = torch.tensor([v_elapsed], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        v_elapsed = float(t.item())
    verified = {"ms_per_step": round(v_elapsed / args.steps * 1e3, 4),
                "value": round(total * args.steps / v_elapsed / 1e9, 3), "unit": "GB/s",
                "records": int(v_out if not use_dist else (v_out.shape[0] if v_out is not None else -1)),
                "what": "scan + compaction + on-device pre-verification (yr_amd_verify_device)"
                        + ("" if not use_dist else " of each rank's window + %s gather of the "
                           "{offset, pool index} records to rank 0"
                           % ("RCCL" if args.backend == "nccl" else args.backend))}

    run(args.warmup)
    for sc in scanners:
        sc.set_timing(True)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pos, kernel_ms = run(args.steps, True)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for sc in scanners:
        sc.set_timing(False)
    per_rank = None
    if use_dist:
        # attribution of an N > 1 step (max over ranks below): every rank's
        # own scan-kernel average (HIP events), its wall time and the wall time
        # it spent in the candidate gathers, so a slow rank and a slow gather
        # are told apart
        mine = torch.tensor([sum(kernel_ms) / len(kernel_ms), min(kernel_ms), max(kernel_ms),
                             elapsed, gather_s[0]], dtype=torch.float64,
                            device=dev if args.backend == "nccl" else "cpu")
        rows = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(rows, mine)
        rows = [r.cpu().tolist() for r in rows]

        def mma(v, nd=4):
            return {"min": round(min(v), nd), "max": round(max(v), nd),
                    "avg": round(sum(v) / len(v), nd), "by_rank": [round(x, nd) for x in v]}
        per_rank = {
            "per_rank_kernel_ms": mma([r[0] for r in rows]),
            "per_rank_kernel_ms_extremes": {"min": round(min(r[1] for r in rows), 4),
                                            "max": round(max(r[2] for r in rows), 4)},
            "per_rank_step_ms": mma([r[3] / args.steps * 1e3 for r in rows]),
            "per_rank_gather_ms_per_step": mma([r[4] / args.steps * 1e3 for r in rows]),
            "what": "per rank over the timed steps: scan-kernel HIP-event average (and the "
                    "extreme single launches), the rank's wall time per step, and its wall time "
                    "per step inside the candidate gather (D2D copy + %s counts all-gather + "
                    "padded gather); scans of later steps are queued behind, so gather time "
                    "overlaps the GPU" % ("RCCL" if args.backend == "nccl" else args.backend)}
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_bytes = total * args.steps
    value = total_bytes / elapsed / 1e9
    k_avg = sum(kernel_ms) / len(kernel_ms)
    achieved = shard / (k_avg * 1e-3) / 1e9

    # parity spot check of this run's own output (rank 0): ascending and the
    # candidate count of config C at 4 GiB recorded from the reference run
    # on-device pre-verification of the last step's candidates (SURVEY.md §8f
    # rows 1 and 4; not part of the timed step): how many of the reference's
    # verify calls can have an effect, and what it costs on the GPU
    preverify = None
    if rank == 0 and world == 1:
        scanner.scan_device(buf.data_ptr(), total)
        scanner.device_result()
        torch.cuda.synchronize()
        scanner.verify_device(0)                    # workspace allocation
        t0 = time.perf_counter()
        _, n_rec = scanner.verify_device(0)
        preverify = {"records": int(n_rec), "ms": round((time.perf_counter() - t0) * 1e3, 3),
                     "what": "verify calls left for the host after on-device literal/hex "
                             "pre-verification of the candidates (yr_amd_verify_device, "
                             "synchronous, wall clock)"}

    check = None
    if rank == 0 and not args.no_check:
        if not use_dist:
            ptr, cnt = pos
            pos = torch.empty(max(cnt, 1), dtype=torch.int64, device=dev)
            memcpy(pos.data_ptr(), ptr, cnt * 8, 3)
            pos = pos[:cnt]
        p = pos.cpu().numpy()
        ok = bool((p[1:] > p[:-1]).all()) if p.size > 1 else True
        check = {"ascending": ok, "candidates": int(p.size)}
        if args.rules == "C" and shard == 4 * GiB and args.seed == 1 and world <= 8:
            # every rank's shard against its golden (tests/golden/config_d.json,
            # shard 0 = the stock golden C_4G): count and SHA-256 of its positions
            import oracle
            with open(os.path.join(REPO, "tests", "golden", "config_d.json")) as f:
                gold = json.load(f)["shards"][:world]
            bounds = [ydist.shard_bounds(total, world, r) for r in range(world)]
            parts = [p[(p > b) & (p <= e)] if b > 0 else p[p <= e] for b, e in bounds]
            check["golden_candidate_count"] = sum(g["count"] for g in gold)
            check["match_golden"] = all(
                q.size == g["count"] and oracle.positions_sha(q) == g["sha"]
                for q, g in zip(parts, gold))
            check["golden"] = ("tests/golden/config_d.json, %d shard(s); shard 0 = stock "
                               "golden C_4G" % world)

    if rank == 0:
        traffic, traffic_src = load_traffic(shard)
        cpu = cpu1 = cpu_par = None
        if world == 1 and not args.no_cpu:
            import oracle
            sample = oracle.xorshift(args.cpu_sample_mib << 20, args.seed)
            info = cpu_info()
            threads = args.cpu_threads or info["affinity"]
            # the CPU comparator: stock libyara on every CPU of the host this
            # process may use (SURVEY.md §8d "nproc threads") and at the CPUs
            # the host actually grants it (min(affinity, ceil(cgroup quota)):
            # a GPU box's cgroup may grant far fewer than it shows); the faster
            # of the two is cpu_baseline.  The 1-thread stock scan and the
            # restatement's slice walkers beside them.
            granted = threads
            if not args.cpu_threads and "cgroup_cpus" in info:
                granted = max(1, min(info["affinity"], int(-(-info["cgroup_cpus"] // 1))))
            cpu_all = cpu_stock_threads(args.rules, sample, args.seed, threads)
            cpu_granted = (cpu_stock_threads(args.rules, sample, args.seed, granted)
                           if granted != threads else None)
            legs = [c for c in (cpu_all, cpu_granted) if c and "value" in c]
            cpu = max(legs, key=lambda c: c["value"]) if legs else cpu_all
            if legs:
                pick = "granted" if cpu is cpu_granted else "affinity"
                cpu = dict(cpu)
                cpu["legs"] = {"affinity": {"threads": threads,
                                            "GB/s": (cpu_all or {}).get("value")},
                               "granted": {"threads": granted, "GB/s": (
                                   cpu_granted or cpu_all or {}).get("value")}}
                cpu["chosen"] = pick + (" (min(affinity, ceil(cgroup CPU quota)) threads)"
                                        if pick == "granted" else " (every CPU in the "
                                        "process's affinity mask)")
            cpu1 = cpu_baseline(args.rules, sample, args.seed)
            cpu_par = cpu_parallel(args.rules, sample, granted)
            if cpu is None:
                cpu, cpu1 = cpu1, None
            del sample
        line = {
            "metric": "scanned GB/s per GPU (4 GiB buffer, 10k atoms) + bit-exact match-set vs CPU",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (SURVEY.md App. A xorshift64 seed %d, generated in HBM)" % args.seed,
            "config": {"workload": "config %s: %d strings -> AC tables of stock libyara 4.2.1, "
                                   "%.0f GiB per GPU%s" % (
                                       args.rules, {"B": 1000, "C": 10000, "E": 2000}.get(args.rules, 0),
                                       args.gib_per_gpu,
                                       "" if not use_dist else ", one %d GiB buffer sharded "
                                       "(shard + verify halos per GPU), RCCL gather of candidate "
                                       "lists" % (args.gib_per_gpu * world)),
                       "bytes_per_gpu": shard, "parallelism": "shard%d" % world,
                       **({"dist_backend": args.backend} if use_dist else {})},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": "scan_segments_kernel", "kernel_ms_avg": round(k_avg, 4)},
            "cpu_baseline": cpu,
            "cpu_baseline_1thread": cpu1,
            "cpu_port_parallel": cpu_par,
            "preverify": preverify,
            "verified_step": verified,
            "check": check,
            "other_rule_sets": other,
        }
        if per_rank is not None:
            line["multi"] = per_rank
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
