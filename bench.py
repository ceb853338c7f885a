"""Benchmark: stories15M batched prefill on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--global-batch G]
    N > 1: either under python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N,
    or plain `python bench.py --gpus N`, which starts the N rank processes itself (spawn_ranks)
    --global-batch G: strong scaling instead (G rows split over the N GPUs; C4 is G = 2048)

One step = one full forward (Llama.__call__ semantics: embedding, 6 blocks, final
norm + lm_head on the last position) of B=256 sequences x L=256 tokens per GPU,
start_pos 0, ids already resident in HBM, logits left in HBM; for N > 1 each rank
owns its 256 batch rows (weak scaling, reference rows are independent:
llama3.py:163-211) and the step ends with the single RCCL gather of every rank's
logits to rank 0 over xGMI (on the context stream, after the forward that wrote the rows).
Rank 0 prints one JSON line.

value: the product forward (layers as two batch-row ranges on two HIP streams,
l3_set_batch_split; the last block's attention / O-proj / FFN on each sequence's last
position, the only rows that reach the logits, l3_set_last_layer_rows — its QKV GEMM still
appends every position to the KV cache), no events in the timed region; beside it
ms_per_step_all_rows_last_layer, the same steps with every position through the last block.
The roofline, per-kernel and C5 passes run every position of every layer.
roofline: the dominant kernel is the fused gate|up GEMM (N = 2*FD = 1536, K = 288,
M = 65,536 rows) — algorithmic FLOPs 2*M*K*N per launch over its mean HIP-event
duration on the context stream, against the 157.3 TFLOP/s dense fp32 MFMA peak, timed in
a second region of the same K steps with the split off (two row ranges in flight share
the CUs, so a launch's duration would not measure the kernel): ms_per_step_serialized.
"ffn" adds the down GEMM (the metric's "% fp32 MFMA peak on FFN GEMM").
traffic: HBM bytes per gate|up launch from the committed rocprofv3 PMC summary
(profiles/pmc_gateup.json, FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction), or null.
cpu_baseline: the oracle (NumPy restatement of the reference, oracle/) timed on
this host's cores on the C3 workload itself (B=256, L=256) per SURVEY 8(d): one warm-up
forward, median of 3; rank 0 at N=1 only.
Host path (ms_per_step_with_logits_d2h): Llama.__call__ on host ids, logits returned in a
pinned NumPy array (l3hip.PinnedPool): ids H2D + forward + logits D2H, never `value`.
N > 1 (or --rccl): after the timed region rank 0 recomputes every peer's seeded id block on
its own context and compares it bit for bit with the gathered rows; a mismatch exits 3.
"""

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "llama3.np_amd"))

import l3hip  # noqa: E402
import llama3  # noqa: E402
import synth  # noqa: E402

METRIC = "tokens/s stories15M batch-256 seq-256 prefill; % fp32 MFMA peak on FFN GEMM"
PEAK_FP32_TFLOPS = 157.3  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
# the x6 path's ceiling in fp32-equivalent FLOP/s: the dense bf16 MFMA peak (256 CUs x 4 SIMDs x
# 1024 FLOP/clk x 2.4 GHz = 2516.6 TF/s, MI355X_MICROARCH.md) over its six products per fp32 one
PEAK_X6_TFLOPS = round(2516.6 / 6, 1)
B_PER_GPU, SEQ = 256, 256


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, cmd=None, timeout_s=1800.0, grace_s=20.0, out=None):
    """``--gpus N`` with no launcher (WORLD_SIZE unset): start N fresh rank processes, one per
    GPU, the way torch.distributed.run would, and wait for them.

    Called before this process makes any GPU call (the ranks are children started with
    subprocess, never exec'd over this process).  Each child gets RANK / LOCAL_RANK /
    WORLD_SIZE / LOCAL_WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free MASTER_PORT and an
    L3_LAUNCH_KEY unique to this launch (the RCCL-id hand-off file, l3hip.launch_key()).
    Rank 0's stdout is this process's stdout (its one JSON line is the bench line); the other
    ranks' stdout goes to stderr.  If any rank fails, the ranks still running are given
    ``grace_s`` and then killed by pid (a peer blocked in an RCCL call never returns on its
    own), and the first failing rank's exit status is returned; 0 when every rank succeeded.
    ``timeout_s`` (default 30 min, ``--spawn-timeout``; None: no limit) bounds the whole launch
    (every rank hung together, e.g. in RCCL init, returns 124).  On any exit path — a
    KeyboardInterrupt or SIGTERM in this process included — every child still running is killed
    by pid and reaped, so no rank is left holding its GPU.
    ``cmd`` (tests) replaces the rank body ``[python, bench.py] + argv``."""
    import signal
    import subprocess
    import uuid

    port = _free_port()
    key = f"spawn_{os.getpid()}_{port}_{uuid.uuid4().hex[:12]}"
    base = list(cmd) if cmd else [sys.executable, "-u", os.path.abspath(__file__)]
    out = sys.stdout if out is None else out
    procs = []

    def _term(signum, frame):  # SIGTERM -> the finally below reaps the ranks
        raise SystemExit(128 + signum)

    old_term = None
    try:
        old_term = signal.signal(signal.SIGTERM, _term)
    except ValueError:  # not the main thread: the finally still covers KeyboardInterrupt
        pass
    first_bad = None
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(port), L3_LAUNCH_KEY=key)
            procs.append(subprocess.Popen(base + list(argv), env=env,
                                          stdout=out if r == 0 else sys.stderr))
        t0 = time.time()
        bad_at = None
        while True:
            rcs = [p.poll() for p in procs]
            for r, rc in enumerate(rcs):
                if rc not in (None, 0) and first_bad is None:
                    first_bad, bad_at = (r, rc), time.time()
            if all(rc is not None for rc in rcs):
                break
            late = timeout_s is not None and time.time() - t0 > timeout_s
            if late or (bad_at is not None and time.time() - bad_at > grace_s):
                if first_bad is None:
                    first_bad = (-1, 124)
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()  # the exact child pid this function started
        for p in procs:
            p.wait()
        if old_term is not None:
            signal.signal(signal.SIGTERM, old_term)
    if first_bad is not None:
        r, rc = first_bad
        print(json.dumps({"error": "rank failed" if r >= 0 else "ranks timed out", "rank": r,
                          "rc": rc, "world": n}), file=sys.stderr, flush=True)
        return rc if isinstance(rc, int) and rc > 0 else 1
    return 0


class Dist:
    """One process per GPU (torch.distributed.run env, or the ranks spawn_ranks started).  No
    PyTorch in this process: the RCCL id goes rank 0 -> peers through an atomically renamed
    file (single node, l3hip.launch_key()), and barriers / the max-over-ranks time run over
    RCCL itself."""

    def __init__(self, n, force_comm=False):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if n != self.world:
            raise SystemExit(f"--gpus {n} but WORLD_SIZE={self.world}")
        self.ctx = None
        self.force_comm = force_comm

    @property
    def comm(self):
        return self.world > 1 or self.force_comm

    def init_comm(self, ctx, overlap=False):
        """Communicator up, then what RCCL saw (ncclCommCount, every rank's PCI bus id gathered
        over RCCL itself): every rank checks it (check_devices), so a run that is not N ranks on
        N distinct GPUs stops on every rank at once, before any timed step."""
        self.ctx = ctx
        self.info = None
        if self.world > 1 or self.force_comm:
            key = l3hip.launch_key()
            uid = l3hip.exchange_unique_id(self.rank, self.world, key)
            ctx.comm_init(self.world, self.rank, uid)
            ctx.comm_barrier()
            if self.rank == 0:  # every rank has read the id once the communicator is up
                l3hip.remove_unique_id(key)
            if overlap:
                ctx.set_comm_overlap(True)
            info = ctx.comm_info()
            self.info = check_devices(info["nranks"], self.world, info["busids"], info["rank"],
                                      self.rank)
            self.info["comm_mode"] = "overlapped" if overlap else "serialized"

    def barrier(self):
        if self.comm:
            self.ctx.comm_barrier()

    def max(self, x):
        return self.ctx.comm_max(x) if self.comm else x

    def min(self, x):
        return -self.ctx.comm_max(-x) if self.comm else x


class SingleProcess:
    """--single-process: this one process drives N GPUs through l3hip.Group (ncclCommInitAll,
    one thread, one grouped gather per step); barriers and max-over-ranks are local."""

    def __init__(self, n):
        if "WORLD_SIZE" in os.environ and os.environ["WORLD_SIZE"] != "1":
            raise SystemExit("--single-process drives every GPU from one process: no launcher")
        self.world, self.rank, self.local_rank, self.comm = n, 0, 0, n > 1
        self.info = None

    def barrier(self):
        pass

    def max(self, x):
        return x

    def min(self, x):
        return x


def check_devices(nranks, world, busids, rank_seen, rank):
    """The N > 1 proof the driver's scaling line needs: RCCL's own rank count equals WORLD_SIZE,
    it numbers this process as RANK, and every rank sits on a distinct PCI device.  Returns the
    fields for the JSON line; raises SystemExit(4) otherwise (every rank sees the same gathered
    list, so every rank stops)."""
    errs = []
    if nranks != world:
        errs.append(f"RCCL counts {nranks} ranks, WORLD_SIZE is {world}")
    if rank_seen != rank:
        errs.append(f"RCCL numbers this process {rank_seen}, RANK is {rank}")
    if len(busids) != nranks:
        errs.append(f"{len(busids)} bus ids for {nranks} ranks")
    dup = sorted({b for b in busids if busids.count(b) > 1})
    if dup:
        errs.append(f"ranks share a device: {dup}")
    if errs:
        print(json.dumps({"error": "multi-GPU device check failed", "details": errs,
                          "rccl_nranks": nranks, "devices": busids}), flush=True)
        raise SystemExit(4)
    return {"rccl_nranks": nranks, "devices": list(busids)}


def cpu_baseline():
    """Oracle (port of the reference's NumPy forward) on the C3 workload itself, SURVEY 8(d):
    B=256, L=256, one warm-up forward, median of 3, OpenBLAS on every thread this process may
    use; plus a 1-thread figure on a labelled sample of the same workload (16 of its 256 rows:
    the rows are independent, llama3.py:163-211, so the rate per row is the C3 rate).

    Thread count: OpenBLAS takes OPENBLAS_NUM_THREADS, else OMP_NUM_THREADS.  The GPU box
    exports OMP_NUM_THREADS=16 — its CPU share per GPU, which its rules say to leave as set —
    so on the box the figure is 16 threads of a 256-CPU host, and the line says so
    (cores / nproc / affinity / thread_cap)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import llama3_oracle as orc

    try:
        from threadpoolctl import threadpool_info

        blas = max([d.get("num_threads", 1) for d in threadpool_info()] or [1])
    except Exception:
        blas = int(os.environ.get("OPENBLAS_NUM_THREADS", os.environ.get("OMP_NUM_THREADS", 1)))
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:
        affinity = None
    cap = None
    for var in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS"):
        if os.environ.get(var):
            cap = f"{var}={os.environ[var]}"
            break
    Bs = B_PER_GPU
    args = synth.stories15m(Bs)
    w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=0)
    model = orc.OracleModel(w, args)
    ids = np.random.default_rng(1).integers(0, args.vocab_size, (Bs, SEQ))
    model(ids, 0)  # warm-up
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        model(ids, 0)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    one, B1 = None, 16
    try:
        from threadpoolctl import threadpool_limits

        with threadpool_limits(limits=1):
            t1 = time.perf_counter()
            model(ids[:B1], 0)
            one = round(B1 * SEQ / (time.perf_counter() - t1), 1)
    except Exception:
        pass
    # "cores" is the contract's name for the threads actually used (one OpenBLAS thread per core
    # it runs on); "threads" says the same under its plain name
    return {"value": round(Bs * SEQ / t, 1), "unit": "tokens/s", "cores": int(blas), "threads": int(blas),
            "nproc": os.cpu_count(), "affinity": affinity, "openblas_threads": int(blas),
            "thread_cap": cap,
            "cores_why": ("all the cores this job may use: the GPU box gives one GPU's job a 16-CPU share "
                          "(it exports OMP_NUM_THREADS=16 and its rules size worker pools to that share); "
                          "nproc / affinity report the whole host, not the share") if cap and cap.endswith("=16")
                         else "OpenBLAS's own thread count on this host",
            "value_1_thread_sample": one,
            "sample_1_thread": f"B={B1} of the C3 batch's {Bs} rows, L={SEQ}, one forward, "
                               f"OpenBLAS limited to 1 thread (rows independent: same per-row work)",
            "kind": "port",
            "sample": f"oracle/llama3_oracle.py (NumPy restatement of the reference, f64 after layer-0 "
                      f"RoPE as the reference) stories15M prefill B={Bs} L={SEQ} (the C3 workload), "
                      f"1 warm-up, median of 3 ({', '.join(f'{x:.2f}' for x in times)} s), "
                      f"OpenBLAS threads={blas} of nproc={os.cpu_count()} "
                      f"(affinity {affinity}; cap: {cap or 'none'})"}


def step_flops(args, FD, B, L, pruned):
    """Algorithmic FLOPs one forward executes (SURVEY 8(d) counts; llama3.py:166-211,97-103,304-307).

    pruned=False: every row through every layer (GEMMs 2*T*K*N each, causal attention
    4*H*HD*B*L(L+1)/2) + the last-position lm_head.  pruned=True: what the product forward runs
    (runtime.hip run_layer(..., last_rows)): the last block computes K / V for every position (the
    cache) and its q, attention (one query per sequence over L keys), O-proj and FFN on each
    sequence's last position only.  C3: 845.68 GFLOP all rows, 727.8 pruned."""
    D, H = args.dim, args.n_heads
    KVH = args.n_kv_heads or H
    HD = D // H
    qdim, kvdim = H * HD, KVH * HD
    T = B * L

    def gemms(rows, qkv_cols):
        return 2.0 * rows * D * (qkv_cols + qdim + 3 * FD) if qkv_cols else 0.0

    full = gemms(T, qdim + 2 * kvdim) + 4.0 * H * HD * B * L * (L + 1) / 2
    lm = 2.0 * B * D * args.vocab_size
    nl = args.n_layers
    if not pruned or L == 1 or nl < 2:
        return nl * full + lm
    last = (2.0 * T * D * 2 * kvdim            # K / V of every position
            + 2.0 * B * D * qdim               # q of the last positions
            + 4.0 * H * HD * B * L             # one query per sequence over L keys
            + 2.0 * B * D * (qdim + 3 * FD))   # O-proj, gate|up, down on B rows
    return (nl - 1) * full + last + lm


def traffic_per_launch(rows, name="pmc_gateup.json"):
    p = os.path.join(REPO, "profiles", name)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    if d.get("workload_rows") != rows or d.get("source_hash") != l3hip.source_hash():
        return None  # counters were measured on another build of the library
    return d.get("hbm_bytes_per_launch")


W_KINDS = {"self_attn.q_proj.weight": l3hip.W_Q, "self_attn.k_proj.weight": l3hip.W_K,
           "self_attn.v_proj.weight": l3hip.W_V, "self_attn.o_proj.weight": l3hip.W_O,
           "mlp.gate_proj.weight": l3hip.W_GATE, "mlp.up_proj.weight": l3hip.W_UP,
           "mlp.down_proj.weight": l3hip.W_DOWN, "input_layernorm.weight": l3hip.W_ATTN_NORM,
           "post_attention_layernorm.weight": l3hip.W_FFN_NORM}


def upload_weights(ctx, w, n_layers):
    """Every tensor of a weight mapping through the C ABI (what Llama.__init__ does from an .npz),
    then finalize."""
    ctx.upload(0, l3hip.W_EMBED, w["model.embed_tokens.weight"])
    for i in range(n_layers):
        for name, kind in W_KINDS.items():
            ctx.upload(i, kind, w[f"model.layers.{i}.{name}"])
    ctx.upload(0, l3hip.W_FINAL_NORM, w["model.norm.weight"])
    ctx.upload(0, l3hip.W_LM_HEAD, w["lm_head.weight"])
    ctx.finalize()


def c5_context(n_layers, B, L):
    """A Llama-3-8B-shaped context (D 4096, H 32 / KVH 8, FD 14336, VS 128256) with synthetic
    weights uploaded tensor by tensor through the C ABI (synth.pool_weights: views of a uniform
    256M-float pool, std 0.02 — an 8.5G-sample normal draw would take minutes)."""
    args = synth.llama3_shape(n_layers=n_layers, max_batch_size=B, max_seq_len=L)
    dims = l3hip.Dims(dim=args.dim, n_layers=args.n_layers, n_heads=args.n_heads,
                      n_kv_heads=args.kv_heads, vocab_size=args.vocab_size,
                      hidden_dim=synth.LLAMA3_HIDDEN, max_seq_len=L, max_batch_size=B,
                      norm_eps=args.norm_eps)
    ctx = l3hip.Context(dims, 0)
    rng = np.random.default_rng(0)
    upload_weights(ctx, synth.pool_weights(args, synth.LLAMA3_HIDDEN, rng=rng), args.n_layers)
    return ctx, args, rng


def bench_c5_decode(a):
    """Greedy decode at the Llama-3-8B shape (32 layers, B = 1): a 64-token prefill, then the
    device loop (generate_all) for a.steps + 2 tokens and the lazy one-step-per-call schedule
    for the same tokens (ids must agree).  Decode streams every weight once per token, so the
    roofline is HBM: weight bytes per token / time per token against 8 TB/s."""
    B, L0 = 1, 64
    ctx, args, rng = c5_context(a.layers, B, 2048)
    D, FD, VS, H, KVH = args.dim, synth.LLAMA3_HIDDEN, args.vocab_size, args.n_heads, args.kv_heads
    HD = D // H
    ids = rng.integers(0, VS, (B, L0))
    n = L0 + max(3, a.steps + 2)
    # L3_DECODE_GRAPH=0 (per-kernel profiling: kernel tracing does not survive capture) has no
    # device loop; only the lazy schedule runs then, eager step by step
    graphs = os.environ.get("L3_DECODE_GRAPH", "1") != "0"
    dev_ids, t_dev, t_head = None, None, None
    if graphs:
        ctx.greedy_generate(ids, L0 + 4)  # warm-up: captures the decode graphs
        # decode steps only: the prefill (64 rows through the MFMA GEMMs) and the eager first
        # step are timed on their own and taken out
        t0 = time.perf_counter()
        ctx.greedy_generate(ids, L0 + 2)
        t_head = time.perf_counter() - t0
        t0 = time.perf_counter()
        dev_ids = ctx.greedy_generate(ids, n)
        t_dev = time.perf_counter() - t0 - t_head
    ctx.set_decode_horizon(n)
    lazy = []
    nxt, _ = ctx.greedy_step(ids, 0)
    lazy.append(int(nxt[0]))
    nxt, _ = ctx.greedy_step(nxt.reshape(1, 1), L0 + 1)
    lazy.append(int(nxt[0]))
    t0 = time.perf_counter()
    for i in range(2, n - L0):
        nxt, _ = ctx.greedy_step(nxt.reshape(1, 1), L0 + i)
        lazy.append(int(nxt[0]))
    t_lazy = time.perf_counter() - t0
    steps = n - L0 - 2
    w_bytes = 4 * (args.n_layers * (D * (H + 2 * KVH) * HD + D * H * HD + 3 * D * FD) + VS * D)
    ms = (t_dev if graphs else t_lazy) / steps * 1e3
    print(json.dumps({
        "metric": "ms/token Llama-3-shape greedy decode B=1 (decode path at a bandwidth-bound size)",
        "value": round(ms, 3), "unit": "ms/token", "higher_is_better": False, "n_gpus": 1,
        "config": {"workload": f"Llama-3-8B shape, {args.n_layers} layers, B=1, prefill {L0}, "
                               f"{steps} timed decode steps (prefill and step 1 excluded)", "seq_len": n},
        "device_loop_ms_per_token": round(ms, 3) if graphs else None,
        "lazy_generate_ms_per_token": round(t_lazy / steps * 1e3, 3),
        "ids_equal_lazy_vs_device_loop": bool(dev_ids[0].tolist() == lazy) if graphs else None,
        "decode_graphs": graphs,
        "prefill_and_step1_ms": round(t_head * 1e3, 3) if graphs else None,
        "roofline": {"bound": "hbm", "achieved": round(w_bytes / (ms * 1e-3) / 1e9, 1),
                     "peak": 8000.0, "unit": "GB/s",
                     "frac": round(w_bytes / (ms * 1e-3) / 1e9 / 8000.0, 4),
                     "traffic": None, "bytes_per_token": w_bytes},
        "lib": {"version": l3hip.version(), "source_hash": l3hip.source_hash()}}))


def bench_c5(a):
    """BASELINE configs[4]: Llama-3-8B-shaped prefill (D 4096, 32 layers, H 32 / KVH 8,
    FD 14336, VS 128256), B=64, L=2048 on one GPU — a roofline report, not the headline line.
    Weights (32 GB fp32) are synthetic and uploaded tensor by tensor through the C ABI
    (uniform with std 0.02 drawn from a 256M-float pool: an 8.5G-sample normal draw would take
    minutes); the forward is the same l3_forward_dev as the headline bench."""
    B, L = 64, 2048
    t_up = time.perf_counter()
    ctx, args, rng = c5_context(a.layers, B, L)
    D, FD, VS, H, KVH = args.dim, synth.LLAMA3_HIDDEN, args.vocab_size, args.n_heads, args.kv_heads
    HD = D // H
    ctx.set_last_layer_rows(True)  # the whole-forward TF/s counts every row of every layer
    t_up = time.perf_counter() - t_up
    ids = rng.integers(0, VS, (B, L)).astype(np.int32)
    ids_dev = ctx.alloc(ids.nbytes)
    ctx.h2d(ids_dev, ids)
    logits_dev = ctx.alloc(B * VS * 4)
    for _ in range(a.warmup):
        ctx.forward_dev(ids_dev, B, L, 0, logits_dev)
    ctx.synchronize()
    ctx.kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctx.forward_dev(ids_dev, B, L, 0, logits_dev)
    ctx.synchronize()
    el = time.perf_counter() - t0
    st = ctx.kernel_stats()
    ctx.kernel_timing(False)
    T = B * L
    # outside the timed region: every logit finite, and row 0 equal to row 0 run alone (B = 1,
    # same layer kernels; the B = 1 lm_head runs the GEMV, another reduction order over K = 4096,
    # hence 1e-5 rather than bit equality — tests/test_gpu_parity.py measured 1.4e-5 at |logit| ~ 4)
    out = np.empty((B, VS), np.float32)
    ctx.d2h(out, logits_dev)
    finite = bool(np.isfinite(out).all())
    ctx.forward_dev(ids_dev, 1, L, 0, logits_dev)  # ids row 0 is the first L ids
    row0 = np.empty((1, VS), np.float32)
    ctx.d2h(row0, logits_dev)
    row_err = float(np.max(np.abs(row0[0].astype(np.float64) - out[0])))
    row_ok = bool(np.allclose(row0[0], out[0], rtol=1e-5, atol=1e-5))
    if not (finite and row_ok):
        print(json.dumps({"error": "c5 output check failed", "finite": finite,
                          "row0_vs_alone_max_abs": row_err}), flush=True)
        raise SystemExit(3)
    flops = {"qkv": 2.0 * T * D * (H + 2 * KVH) * HD, "oproj": 2.0 * T * D * D,
             "gateup": 2.0 * T * D * 2 * FD, "down": 2.0 * T * FD * D,
             "attn": 4.0 * HD * H * B * L * (L + 1) / 2, "lmhead": 2.0 * B * D * VS}
    total = args.n_layers * sum(v for k, v in flops.items() if k != "lmhead") + flops["lmhead"]
    per = {k: {"ms": round(st[k][0] / st[k][1], 3),
               "TFLOP/s": round(flops[k] / (st[k][0] / st[k][1] / 1e3) / 1e12, 1)}
           for k in flops if st[k][1]}
    gu = per["gateup"]["TFLOP/s"]
    x6 = None
    if not a.no_x6:
        # beside the line: the opt-in x6 GEMM path (l3_set_gemm_x6) on the same forward, its
        # logits against the fp32 path's (the pieces need 1.5x the layer weights: 42 GB here)
        ctx.forward_dev(ids_dev, B, L, 0, logits_dev)  # the fp32 logits of the whole batch again
        ctx.d2h(out, logits_dev)
        ctx.set_gemm_x6(True)
        ctx.forward_dev(ids_dev, B, L, 0, logits_dev)
        ctx.synchronize()
        ctx.kernel_timing(True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ctx.forward_dev(ids_dev, B, L, 0, logits_dev)
        ctx.synchronize()
        el6 = time.perf_counter() - t0
        st6 = ctx.kernel_stats()
        ctx.kernel_timing(False)
        o6 = np.empty((B, VS), np.float32)
        ctx.d2h(o6, logits_dev)
        ctx.set_gemm_x6(False)
        per6 = {k: {"ms": round(st6[k][0] / st6[k][1], 3),
                    "TFLOP/s (fp32-equivalent)": round(flops[k] / (st6[k][0] / st6[k][1] / 1e3) / 1e12, 1)}
                for k in flops if st6[k][1]}
        gu6 = per6["gateup"]["TFLOP/s (fp32-equivalent)"]
        x6 = {"value": round(T * a.steps / el6, 1), "unit": "tokens/s", "ms_per_step": round(el6 / a.steps * 1e3, 1),
              "whole_forward_fp32_equivalent_TFLOP/s": round(total * a.steps / el6 / 1e12, 1),
              "logits_max_abs_diff_vs_fp32_path": float(np.abs(o6 - out).max()),
              "argmax_rows_equal_vs_fp32_path": f"{int((o6.argmax(1) == out.argmax(1)).sum())}/{B}",
              "roofline": {"kernel": "x6 gemm gate|up, M=131072 K=4096 N=28672", "bound": "mfma",
                           "achieved": gu6, "peak": PEAK_X6_TFLOPS,
                           "unit": "fp32-equivalent TFLOP/s (6 bf16 MFMA per fp32 product)",
                           "frac": round(gu6 / PEAK_X6_TFLOPS, 4),
                           "vs_fp32_mfma_peak": round(gu6 / PEAK_FP32_TFLOPS, 4)},
              "kernels": per6}
    print(json.dumps({
        "metric": "tokens/s Llama-3-shape prefill B=64 L=2048 (roofline report, BASELINE configs[4])",
        "value": round(T * a.steps / el, 1), "unit": "tokens/s", "n_gpus": 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 1), "higher_is_better": True,
        "dtype": "fp32", "data": "synthetic uniform weights (std 0.02), uniform random ids",
        "config": {"workload": f"Llama-3-8B shape, {args.n_layers} layers, B=64 L=2048",
                   "global_batch": B, "seq_len": L},
        "whole_forward_TFLOP/s": round(total * a.steps / el / 1e12, 1),
        "whole_forward_frac": round(total * a.steps / el / 1e12 / PEAK_FP32_TFLOPS, 4),
        "roofline": {"kernel": "gemm gate|up, M=131072 K=4096 N=28672", "bound": "mfma",
                     "achieved": gu, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(gu / PEAK_FP32_TFLOPS, 4),
                     "traffic": traffic_per_launch(T, "pmc_c5_gateup.json")},
        "kernels": per, "weight_upload_s": round(t_up, 1),
        "output_check": {"all_finite": finite, "row0_vs_B1_run_max_abs": row_err, "tol": "1e-5 abs+rel"},
        "gemm_x6": x6,
        "lib": {"version": l3hip.version(), "source_hash": l3hip.source_hash()}}))


def cpu_c5_slice():
    """BASELINE.md / SURVEY 8(d): the reference's CPU path on C5 is infeasible in full, so the
    oracle (NumPy restatement, f64 after layer-0 RoPE) is timed on a 2-layer Llama-3-shape slice
    at B = 1, L = 2048 on this host and extrapolated x16 layers x64 sequences (labelled so)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import llama3_oracle as orc

    args = synth.llama3_shape(n_layers=2, max_batch_size=1, max_seq_len=2048)
    t_gen = time.perf_counter()
    w = synth.make_weights(args, synth.LLAMA3_HIDDEN, seed=0)
    t_gen = time.perf_counter() - t_gen
    model = orc.OracleModel(w, args)
    ids = np.random.default_rng(1).integers(0, args.vocab_size, (1, 2048))
    t0 = time.perf_counter()
    out = model(ids, 0)
    t = time.perf_counter() - t0
    assert np.isfinite(out).all()
    full_s = t * (32 / 2) * 64
    try:
        from threadpoolctl import threadpool_info

        cores = max([d.get("num_threads", 1) for d in threadpool_info()] or [1])
    except Exception:
        cores = os.cpu_count() or 1
    print(json.dumps({
        "metric": "CPU baseline, Llama-3-shape prefill B=64 L=2048 (BASELINE configs[4]), extrapolated",
        "slice": "oracle, 2 of 32 layers, B=1, L=2048, one forward", "slice_s": round(t, 2),
        "extrapolated_full_s": round(full_s, 0), "value": round(64 * 2048 / full_s, 2),
        "unit": "tokens/s", "kind": "port", "cores": int(cores), "weight_gen_s": round(t_gen, 1)}))


def check_gathered(ctx, dist, bpg, VS, gathered_dev):
    """N > 1 self-check (untimed): rank 0 recomputes each peer's seeded id block (the same
    default_rng(100 + r) draw the peer used) on its own context — same B, same kernels, so the
    rows must be bit-identical — and compares them with the rows the RCCL gather delivered.
    Returns the number of ranks checked; raises SystemExit(3) on a mismatch."""
    if dist.rank != 0:
        return None
    got = np.empty((bpg * dist.world, VS), np.float32)
    ctx.d2h(got, gathered_dev)  # joins the comm stream: the last gather has landed
    ids_dev = ctx.alloc(bpg * SEQ * 4)
    out_dev = ctx.alloc(bpg * VS * 4)
    want = np.empty((bpg, VS), np.float32)
    try:
        for r in range(dist.world):
            ids = np.random.default_rng(100 + r).integers(0, VS, (bpg, SEQ)).astype(np.int32)
            ctx.h2d(ids_dev, ids)
            ctx.forward_dev(ids_dev, bpg, SEQ, 0, out_dev)
            ctx.d2h(want, out_dev)
            blk = got[r * bpg:(r + 1) * bpg]
            if not np.array_equal(blk, want):
                bad = np.argwhere(blk != want)
                print(json.dumps({"error": "gathered logits differ from rank 0's recomputation",
                                  "rank": r, "mismatches": int(bad.shape[0]),
                                  "first": bad[0].tolist()}), flush=True)
                raise SystemExit(3)
    finally:
        ctx.free(ids_dev)
        ctx.free(out_dev)
    return dist.world


def check_gathered_group(ctx, N, bpg, VS, gathered_dev, ids_blk):
    """--single-process self-check (untimed): member r's rows (global rows r, r + N, ...) of the
    last gathered step against member 0's own recomputation of member r's id block — same B,
    same kernels, so bit-identical.  Returns N; SystemExit(3) on a mismatch."""
    got = np.empty((bpg * N, VS), np.float32)
    ctx.d2h(got, gathered_dev)
    ids_dev = ctx.alloc(bpg * SEQ * 4)
    out_dev = ctx.alloc(bpg * VS * 4)
    want = np.empty((bpg, VS), np.float32)
    try:
        for r in range(N):
            ctx.h2d(ids_dev, ids_blk[r])
            ctx.forward_dev(ids_dev, bpg, SEQ, 0, out_dev)
            ctx.d2h(want, out_dev)
            blk = got[r::N]
            if not np.array_equal(blk, want):
                bad = np.argwhere(blk != want)
                print(json.dumps({"error": "gathered logits differ from member 0's recomputation",
                                  "member": r, "mismatches": int(bad.shape[0]),
                                  "first": bad[0].tolist()}), flush=True)
                raise SystemExit(3)
    finally:
        ctx.free(ids_dev)
        ctx.free(out_dev)
    return N


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-breakdown", action="store_true",
                    help="skip the untimed all-kernel event pass (profiling runs)")
    ap.add_argument("--workload", choices=["c3", "c5", "c5cpu", "c5decode"], default="c3",
                    help="c3: headline stories15M B=256 L=256 (default); c5: Llama-3-shape report; "
                         "c5cpu: the oracle on a 2-layer C5 slice, extrapolated; c5decode: "
                         "Llama-3-shape batch-1 greedy decode (HBM roofline)")
    ap.add_argument("--layers", type=int, default=32, help="c5 only")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="strong scaling: this many rows split over the GPUs (default: 256 per GPU)")
    ap.add_argument("--split", type=int, default=None,
                    help="batch-split parts of the timed forward (default: the library's, 2)")
    ap.add_argument("--no-step-gather", action="store_true",
                    help="diagnostic: communicator up but no gather inside the timed steps")
    ap.add_argument("--rccl", action="store_true",
                    help="communicator, gather and self-check even at N=1 (rehearses the N>1 path "
                         "under torch.distributed.run --nproc-per-node 1)")
    ap.add_argument("--single-process", action="store_true",
                    help="one process drives all N GPUs (l3hip.Group: ncclCommInitAll, one thread, "
                         "one grouped RCCL gather per step) instead of one process per GPU")
    ap.add_argument("--comm-overlap", action="store_true",
                    help="the overlapped gather (l3_comm_set_overlap): the next step's second batch "
                         "part runs during the gather (default: serialized)")
    ap.add_argument("--spawn-timeout", type=float, default=1800.0,
                    help="seconds before spawned ranks still running are killed (0: no limit)")
    ap.add_argument("--no-x6", action="store_true",
                    help="skip the beside-value pass of the opt-in x6 GEMM path (l3_set_gemm_x6)")
    ap.add_argument("--spawn", action="store_true",
                    help="start the rank processes here even at N=1 (rehearses the launcher-free "
                         "N>1 path; N>1 without WORLD_SIZE spawns anyway)")
    a = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and (a.gpus > 1 or a.spawn) and not a.single_process:
        # no launcher: this process only starts the ranks (nothing here has touched the GPU)
        argv = [x for x in sys.argv[1:] if x != "--spawn"]
        raise SystemExit(spawn_ranks(a.gpus, argv, timeout_s=a.spawn_timeout or None))
    if a.workload == "c5":
        return bench_c5(a)
    if a.workload == "c5cpu":
        return cpu_c5_slice()
    if a.workload == "c5decode":
        return bench_c5_decode(a)

    dist = SingleProcess(a.gpus) if a.single_process else Dist(a.gpus, force_comm=a.rccl)
    # default: weak scaling, B = 256 rows per GPU (N = 8 is C4's B = 2048); --global-batch G:
    # strong scaling, G rows split over the N GPUs (C4 at any N)
    if a.global_batch:
        if a.global_batch % dist.world:
            raise SystemExit(f"--global-batch {a.global_batch} not divisible by {dist.world} GPUs")
        bpg = a.global_batch // dist.world
    else:
        bpg = B_PER_GPU
    N = dist.world
    dev = dist.local_rank
    # a launcher that shows each rank only its own GPU (HIP_VISIBLE_DEVICES per rank): that GPU
    # is device 0 here (check_devices still proves N distinct devices over RCCL)
    if not a.single_process and dev > 0 and dev >= l3hip.device_count():
        dev = 0
    args = synth.stories15m(bpg)
    FD, D = synth.STORIES15M_HIDDEN, args.dim
    weights = synth.make_weights(args, FD, seed=0)
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "stories15m_synth.npz")
        synth.save_npz(path, weights)
        if a.single_process:  # one process, N devices: l3hip.Group under Llama(devices=...)
            model = llama3.Llama(path, synth.stories15m(bpg * N), devices=list(range(N)))
        else:
            model = llama3.Llama(path, args, device=dev)
    ctx = model.context
    members = model.group.members if a.single_process else [ctx]
    VS = args.vocab_size

    # inputs resident in HBM before the timed region: rank (member) r's rows are the seeded
    # block default_rng(100 + r); single-process: member r holds global rows r, r + N, ...
    ids_blk = [np.random.default_rng(100 + r).integers(0, VS, (bpg, SEQ)).astype(np.int32)
               for r in (range(N) if a.single_process else [dist.rank])]
    ids_devs = []
    for m, blk in zip(members, ids_blk):
        ids_devs.append(m.alloc(blk.nbytes))
        m.h2d(ids_devs[-1], blk)
    ids_dev = ids_devs[0]
    logits_dev = ctx.alloc(bpg * VS * 4)
    gathered_dev = None
    rows = [bpg] * N
    if not a.single_process:
        dist.init_comm(ctx, overlap=a.comm_overlap)
    if dist.comm and dist.rank == 0:
        gathered_dev = ctx.alloc(bpg * N * VS * 4)
    step_gather = dist.comm and not a.no_step_gather

    if a.single_process:
        info = [m.comm_info(gather_busids=False) for m in members]
        busids = members[0].comm_info()["busids"]
        for r, x in enumerate(info):
            check_devices(x["nranks"], N, busids, x["rank"], r)
        dist.info = {"rccl_nranks": info[0]["nranks"], "devices": busids,
                     "comm_mode": "single-process group (ncclCommInitAll, one thread)"}

        def step():
            if N > 1:
                model.group.forward_dev(ids_devs, bpg * N, SEQ, 0, gathered_dev)
            else:
                ctx.forward_dev(ids_dev, bpg, SEQ, 0, logits_dev)

        sync = model.group.synchronize
    else:
        def step():
            ctx.forward_dev(ids_dev, bpg, SEQ, 0, logits_dev)
            if step_gather:
                ctx.gather_logits(logits_dev, gathered_dev, rows, root=0)

        sync = ctx.synchronize

    def each(fn):
        for m in members:
            fn(m)

    if a.split is not None:
        each(lambda m: m.set_batch_split(a.split))

    def timed_steps(steps):
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        sync()
        el = time.perf_counter() - t0
        dist.barrier()
        return dist.max(el), dist.min(el)

    for _ in range(a.warmup):
        step()
    sync()
    # value: the product forward (batch split into row ranges on concurrent streams), no events
    elapsed, elapsed_min = timed_steps(a.steps)

    # beside `value` (BASELINE.md's plan: the median step): the same steps one at a time, each
    # bracketed by a device sync — the median of those, whose gaps the back-to-back mean hides
    per_step = []
    for _ in range(a.steps):
        sync()
        t0 = time.perf_counter()
        step()
        sync()
        per_step.append(time.perf_counter() - t0)
    median_ms = dist.max(float(np.median(per_step))) * 1e3

    # N > 1: the gathered rows against rank 0's own recomputation (untimed)
    if a.single_process:
        checked = check_gathered_group(ctx, N, bpg, VS, gathered_dev, ids_blk) if N > 1 else None
    else:
        checked = check_gathered(ctx, dist, bpg, VS, gathered_dev) if step_gather else None
    dist.barrier()

    # beside `value`: the same K steps with the last block run on every position (the product
    # runs its attention / O-proj / FFN on each sequence's last position only: the rows that
    # reach the logits; l3_set_last_layer_rows) — and every pass below counts full layers
    each(lambda m: m.set_last_layer_rows(True))
    step()
    elapsed_all_rows, _ = timed_steps(a.steps)

    # roofline: the same K steps serialized (one row range, one stream) with HIP events around
    # the FFN GEMM launches only (12 per step) — with concurrent row ranges two kernels share
    # the CUs and a launch's duration no longer measures that kernel
    each(lambda m: m.set_batch_split(1))
    step()
    ctx.kernel_timing(True, ["gateup", "down"])
    elapsed_serial, _ = timed_steps(a.steps)
    stats = ctx.kernel_stats()
    ctx.kernel_timing(False)
    each(lambda m: m.set_batch_split(a.split if a.split is not None else 2))
    each(lambda m: m.set_last_layer_rows(False))

    # beside `value`: the opt-in x6 GEMM path (l3_set_gemm_x6: the prefill projections from six
    # bf16 MFMA products per fp32 product, gemm_x6.h) on the same steps, its gate|up launch time
    # from a serialized event pass, and its logits against the fp32 path's (never `value`)
    x6 = None
    if not a.no_x6:
        ref_logits = np.empty((bpg, VS), np.float32)
        ctx.d2h(ref_logits, logits_dev)  # the fp32 path's last step (same ids every step)
        each(lambda m: m.set_gemm_x6(True))
        for _ in range(a.warmup):
            step()
        x6_elapsed, _ = timed_steps(a.steps)
        x6_logits = np.empty((bpg, VS), np.float32)
        ctx.d2h(x6_logits, logits_dev)
        each(lambda m: m.set_last_layer_rows(True))
        each(lambda m: m.set_batch_split(1))
        step()
        ctx.kernel_timing(True, ["gateup", "down"])
        timed_steps(a.steps)
        x6_stats = ctx.kernel_stats()
        ctx.kernel_timing(False)
        each(lambda m: m.set_batch_split(a.split if a.split is not None else 2))
        each(lambda m: m.set_last_layer_rows(False))
        each(lambda m: m.set_gemm_x6(False))
        x6 = (x6_elapsed, x6_stats, float(np.abs(x6_logits - ref_logits).max()),
              int((x6_logits.argmax(1) == ref_logits.argmax(1)).sum()))

    # N > 1: the logits gather alone (untimed for `value`): its share of a step at this N,
    # which the overlapped gather hides behind the next step's layers
    gather_ms = None
    if dist.comm and not a.single_process:
        dist.barrier()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ctx.gather_logits(logits_dev, gathered_dev, rows, root=0)
        ctx.synchronize()
        gather_ms = dist.max(time.perf_counter() - t0) / a.steps * 1e3

    # the drop-in host path, Llama.__call__ on host ids (int64) returning host
    # logits (a pinned NumPy array): ids H2D + forward + logits D2H (PCIe-inclusive; reported
    # beside `value`, never as it)
    if a.single_process:  # the global batch: row r + N*j is member r's row j
        ids_host = np.empty((bpg * N, SEQ), np.int64)
        for r, blk in enumerate(ids_blk):
            ids_host[r::N] = blk
    else:
        ids_host = ids_blk[0].astype(np.int64)
    d2h_steps = max(1, min(a.steps, 10))
    out = model(ids_host, 0)
    del out
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(d2h_steps):
        out = model(ids_host, 0)
        del out
    elapsed_d2h = dist.max(time.perf_counter() - t0)

    # sanity on the output (outside the timed region)
    probe = np.empty((2, VS), np.float32)
    ctx.d2h(probe, gathered_dev if a.single_process and N > 1 else logits_dev)
    if not np.isfinite(probe).all():
        raise SystemExit("non-finite logits")

    if dist.rank != 0:
        return
    tokens = bpg * SEQ * dist.world * a.steps
    T = bpg * SEQ
    gu_ms, gu_n = stats["gateup"]
    dn_ms, dn_n = stats["down"]
    gu_flops = 2.0 * T * D * 2 * FD
    dn_flops = 2.0 * T * FD * D
    gu_avg_s = gu_ms / gu_n / 1e3
    achieved = gu_flops / gu_avg_s / 1e12
    ffn_tf = (gu_flops + dn_flops) / ((gu_ms / gu_n + dn_ms / dn_n) / 1e3) / 1e12
    traffic = traffic_per_launch(T)
    host_ms = elapsed_d2h / d2h_steps * 1e3
    # the whole step against the MFMA peak: the FLOPs the timed (pruned) step executes over its
    # wall time, and the all-rows step's full algorithmic count over its own time
    fl_pruned = step_flops(args, FD, bpg, SEQ, True)
    fl_all = step_flops(args, FD, bpg, SEQ, False)
    tf_step = fl_pruned * a.steps / elapsed / 1e12
    tf_all = fl_all * a.steps / elapsed_all_rows / 1e12
    whole_step = {"executed_gflop": round(fl_pruned / 1e9, 2), "achieved": round(tf_step, 2),
                  "frac": round(tf_step / PEAK_FP32_TFLOPS, 4),
                  "all_rows": {"gflop": round(fl_all / 1e9, 2), "achieved": round(tf_all, 2),
                               "frac": round(tf_all / PEAK_FP32_TFLOPS, 4)},
                  "unit": "TFLOP/s", "peak": PEAK_FP32_TFLOPS,
                  "note": "per GPU; executed = the timed step's own work (last block on each sequence's "
                          "last position, step_flops in bench.py), wall clock of the same steps as value"}
    out = {
        "metric": METRIC,
        "value": round(tokens / elapsed, 1),
        "unit": "tokens/s",
        "n_gpus": dist.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "timing": (f"value and ms_per_step: wall clock of {a.steps} back-to-back steps after {a.warmup} "
                   "warm-up steps, bracketed by a barrier and a device sync, max over ranks, mean per step; "
                   "ms_per_step_median: the median of the same steps run one at a time, each between syncs"),
        "ms_per_step_median": round(median_ms, 4),
        "ms_per_step_serialized": round(elapsed_serial / a.steps * 1e3, 4),
        "ms_per_step_all_rows_last_layer": round(elapsed_all_rows / a.steps * 1e3, 4),
        "batch_split": a.split if a.split is not None else 2,
        "ms_per_step_with_logits_d2h": round(host_ms, 4),
        "host_path_tokens_per_s": round(T * dist.world * d2h_steps / elapsed_d2h, 1),
        "ms_per_step_rank_min": round(elapsed_min / a.steps * 1e3, 4),
        "ms_per_step_rank_max": round(elapsed / a.steps * 1e3, 4),
        "launcher": "single-process" if a.single_process else (
            "spawned" if os.environ.get("L3_LAUNCH_KEY", "").startswith("spawn_") else
            "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else "none"),
        "ms_gather_alone": None if gather_ms is None else round(gather_ms, 4),
        "gather_self_check_ranks": checked,
        "higher_is_better": True,
        "scaling": "strong" if a.global_batch else "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic: stories15M-shaped N(0,0.02^2) weights (seed 0), uniform random ids",
        "config": {"workload": f"stories15M prefill, B={bpg} per GPU x L={SEQ}, start_pos 0",
                   "global_batch": bpg * dist.world, "seq_len": SEQ,
                   "parallelism": f"dp{dist.world} (batch rows) + RCCL logits gather"},
        "lib": {"version": l3hip.version(), "source_hash": l3hip.source_hash()},
        **(dist.info or {}),
        "whole_step": whole_step,
        "roofline": {"kernel": f"gemm gate|up (fused SwiGLU epilogue), M={T} K=288 N=1536",
                     "pass": "same workload and step count, batch split off (HIP events need "
                             "the kernel alone on the CUs)",
                     "bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_FP32_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                     "traffic": traffic,
                     "ffn": {"achieved": round(ffn_tf, 2),
                             "frac": round(ffn_tf / PEAK_FP32_TFLOPS, 4)}},
    }
    if x6 is not None:
        x6_elapsed, x6_stats, x6_diff, x6_same = x6
        gu6_ms, gu6_n = x6_stats["gateup"]
        dn6_ms, dn6_n = x6_stats["down"]
        gu6 = gu_flops / (gu6_ms / gu6_n / 1e3) / 1e12
        ffn6 = (gu_flops + dn_flops) / ((gu6_ms / gu6_n + dn6_ms / dn6_n) / 1e3) / 1e12
        out["gemm_x6"] = {
            "what": "opt-in path (l3_set_gemm_x6 / L3_GEMM_X6=1): QKV / O-proj / gate|up / down from "
                    "six bf16 MFMA products per fp32 product (operands cut exactly into three bf16 "
                    "pieces; gemm_x6.h); attention and lm_head fp32; same steps and timing as value",
            "value": round(tokens / x6_elapsed, 1), "unit": "tokens/s",
            "ms_per_step": round(x6_elapsed / a.steps * 1e3, 4),
            "logits_max_abs_diff_vs_fp32_path": x6_diff,
            "argmax_rows_equal_vs_fp32_path": f"{x6_same}/{bpg}",
            "whole_step_fp32_equivalent_tflops": round(fl_pruned * a.steps / x6_elapsed / 1e12, 2),
            "roofline": {"kernel": f"x6 gemm gate|up (fused SwiGLU epilogue), M={T} K=288 N=1536",
                         "bound": "mfma", "achieved": round(gu6, 2), "peak": PEAK_X6_TFLOPS,
                         "unit": "fp32-equivalent TFLOP/s (6 bf16 MFMA per fp32 product)",
                         "frac": round(gu6 / PEAK_X6_TFLOPS, 4),
                         "traffic": traffic_per_launch(T, "pmc_x6_gateup.json"),
                         "bf16_mfma_tflops_executed": round(6 * gu6, 1),
                         "vs_fp32_mfma_peak": round(gu6 / PEAK_FP32_TFLOPS, 4),
                         "ffn": {"achieved": round(ffn6, 2), "frac": round(ffn6 / PEAK_X6_TFLOPS, 4)}},
        }
    if dist.world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    if dist.world == 1 and not a.no_kernel_breakdown:
        # per-kernel breakdown from a separate (untimed, serialized) pass with all events on
        ctx.set_batch_split(1)
        ctx.set_last_layer_rows(True)  # every launch of a kind full size
        ctx.kernel_timing(True)
        for _ in range(3):
            step()
        sync()
        out["kernel_ms"] = {k: round(v[0] / v[1], 4) for k, v in ctx.kernel_stats().items() if v[1]}
        ctx.kernel_timing(False)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
