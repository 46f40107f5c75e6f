"""bench.py -- BASELINE.json metric: env steps/s at N=65536 parallel envs on
pointmaze-large (pointmaze-large-navigate-v0), 1/2/4/8 MI355X.

    python bench.py --gpus N --steps K --warmup W [--workload pointmaze|powder|gcsample]

A step = one ``env.step(action)`` of all envs of this rank: one launch of
``maze_step_kernel`` through the C-ABI (Python -> ctypes -> libogbx), with the
[N,2] float32 actions already resident in HBM (pre-generated ring, seed 1) and
same-step auto-reset.  Timed region: barrier + synchronize, K steps,
synchronize (clock read), barrier; the max over ranks is reported.

Multi-GPU (the metric: N = 65,536 envs in total on 1/2/4/8 GPUs): one process
per GPU; env i lives on rank i // (N/G) (``ogbench_amd.sharding``), each rank's
handle is created at its global ``env_base`` with the one shared seed, so the
G-rank job is the single-GPU job bit for bit (tests/test_shard_gpu.py).  No
data-path collective; ``value`` = N x steps / time -> "scaling": "strong".
The weak-scaling rate (65,536 envs per GPU) is reported in ``extra``.

Launch: under torchrun (WORLD_SIZE set) each process is one rank; a plain
``python bench.py --gpus N`` (N > 1, no WORLD_SIZE) starts the N rank
processes itself before any HIP call and exits with the worst rank status.
A WORLD_SIZE that differs from --gpus, or more nccl (RCCL) ranks than visible
GPUs, is refused (exit 2).  ``ranks_seen`` counts the ranks an untimed
all-gather reached.

Extra fields (not ``value``): the same workload replayed from a hipGraph and
as K fused steps per launch; ``roofline`` of maze_step_kernel (algorithmic
87 B per env-step) from the smaller of two HIP event spans on the
launch stream (the timed region / its steps, >= 1000 back-to-back launches /
count; the per-launch event-pair median beside them); ``cpu_baseline`` = the oracle C restatement
(OpenMP) on a bounded sample.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


class LaunchError(SystemExit):
    """A rank layout bench.py refuses to run (exit status 2, message on stderr)."""

    def __init__(self, msg):
        print(f'bench.py: {msg}', file=sys.stderr, flush=True)
        super().__init__(2)


def _check_world(gpus, backend, env=None):
    """Validate the requested rank layout before anything touches the GPU.

    Returns 'self-launch' when `--gpus N > 1` runs without a launcher (no
    WORLD_SIZE in the environment), 'rank' otherwise.  Raises LaunchError when
    the launcher's WORLD_SIZE differs from --gpus, or when the nccl (RCCL)
    backend is asked for more ranks than there are visible GPUs (one rank per
    GPU; the gloo backend rehearses N ranks on fewer GPUs).  Counting devices
    does not initialise HIP on this image, so this is safe in the parent."""
    env = os.environ if env is None else env
    if gpus < 1:
        raise LaunchError(f'--gpus must be >= 1, got {gpus}')
    ws = env.get('WORLD_SIZE')
    if ws is not None and int(ws) != gpus:
        raise LaunchError(f'--gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks; '
                          f'run with --gpus {ws} or launch {gpus} ranks')
    if backend == 'nccl':
        ndev = torch.cuda.device_count()
        if gpus > ndev:
            raise LaunchError(f'--gpus {gpus} with the nccl (RCCL) backend needs {gpus} visible GPUs, found {ndev} '
                              "(use --dist-backend gloo to rehearse several ranks on fewer GPUs)")
    return 'self-launch' if ws is None and gpus > 1 else 'rank'


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _self_launch(gpus, argv):
    """`bench.py --gpus N` with no launcher: start N rank processes of this
    same command (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on
    127.0.0.1), wait for all of them and return the worst exit status.  The
    parent never touches the GPU; rank 0 prints the one JSON line."""
    import subprocess

    port = str(_free_port())
    procs = []
    for r in range(gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rcs = [p.wait() for p in procs]
    # a rank killed by signal s reports -s; the shell's 128 + s convention
    return max((128 - rc if rc < 0 else rc) for rc in rcs), rcs


def _dist_init(backend='nccl'):
    """One process per GPU.  backend 'nccl' is RCCL; 'gloo' (with ranks sharing
    GPUs: device = LOCAL_RANK mod device count) rehearses the N>1 path on a
    one-GPU box."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    ndev = max(1, torch.cuda.device_count())
    dev_index = local % ndev if backend == 'gloo' else local
    torch.cuda.set_device(dev_index)
    if world > 1:
        import torch.distributed as dist

        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev_index))
        else:
            dist.init_process_group(backend)
    return world, rank, dev_index


def _barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def _max_over_ranks(x, world, dev):
    if world == 1:
        return x
    import torch.distributed as dist

    on_dev = dist.get_backend() == 'nccl'
    t = torch.tensor([x], dtype=torch.float64, device=dev if on_dev else 'cpu')
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _ranks_seen(world, dev):
    """Untimed: the number of distinct ranks an all-gather over the process
    group reaches (1 without one): the line's proof that its n_gpus ranks ran."""
    if world == 1:
        return 1
    import torch.distributed as dist

    on_dev = dist.get_backend() == 'nccl'
    mine = torch.tensor([dist.get_rank()], dtype=torch.int64, device=dev if on_dev else 'cpu')
    got = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(got, mine)
    return len({int(t.item()) for t in got})


def _timed(fn, steps, world, dev, span=None):
    """Wall time of `steps` calls between barrier + synchronize on both sides,
    max over ranks.  span (a list): receives the device time of the same
    region from a HIP event pair on the launch stream, in ms.

    Each rank's clock runs from the end of the leading barrier + synchronize
    to the end of its own trailing synchronize; the trailing barrier follows
    the clock read, so the job time (max over ranks) covers every rank's K
    steps but not the barrier's own collective latency (tens of us over
    RCCL, comparable to 20 steps of a 12-us launch)."""
    _barrier(world)
    torch.cuda.synchronize(dev)
    if span is not None:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(torch.cuda.current_stream(dev))
    t0 = time.perf_counter()
    for i in range(steps):
        fn(i)
    if span is not None:
        b.record(torch.cuda.current_stream(dev))
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    _barrier(world)
    if span is not None:
        span.append(a.elapsed_time(b))
    return _max_over_ranks(dt, world, dev)


def _per_launch_ms(fn, launches, dev, host_us=120.0):
    """Average device duration of one launch: `launches` launches queued back
    to back between one HIP event pair on the stream the kernel runs on
    (torch's current stream), divided by the count.

    A spin kernel (torch.cuda._sleep) is queued first, long enough for the host
    to enqueue every launch behind it, so the span covers the kernels (and the
    dispatch gaps between them), not the host's launch rate (a host-bound call
    such as GCDataset.sample(1024) would otherwise read as its host time)."""
    stream = torch.cuda.current_stream(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(int(launches * host_us * 1e-6 * 2.4e9))
    a.record(stream)
    for i in range(launches):
        fn(i)
    b.record(stream)
    torch.cuda.synchronize(dev)
    return a.elapsed_time(b) / launches


def _host_us_per_call(fn, calls, dev):
    """Host time of one call of `fn` (Python + ctypes + the HIP launch) with
    the device held by a spin kernel, so that no call waits on the GPU: the
    host-side bound on the call rate, reported beside the device time."""
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(int(calls * 60e-6 * 2.4e9))
    t0 = time.perf_counter()
    for i in range(calls):
        fn(i)
    dt = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    return dt / calls * 1e6


def _median_launch_ms(fn, launches, dev, host_us=60.0):
    """Median of per-launch HIP event pairs on the launch stream (torch's
    current stream, which libogbx launches on) around each of `launches`
    launches, queued behind a spin kernel so that they run back to back.  Each
    pair also spans the event packets' own completion overhead (~2 us on
    gfx950), so this over-states a short kernel; reported beside
    _launch_ms's span figure, not used for the roofline."""
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(int(launches * host_us * 1e-6 * 2.4e9))
    for i, (a, b) in enumerate(ev):
        a.record(stream)
        fn(i)
        b.record(stream)
    torch.cuda.synchronize(dev)
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def _launch_ms(span_ms, steps, fn, launches, dev):
    """Per-launch device time for the roofline.  Two upper bounds
    on the kernel's duration, both on the launch stream, both including the
    dispatch gap to the next launch:
      * the HIP event span around the timed region itself / its steps (exactly
        the timed states; never above ms_per_step, but it also counts any host
        launch gaps of a host-bound call such as GCDataset.sample(1024));
      * `launches` (>= 1000) back-to-back launches queued behind a spin kernel
        in one event span / count (device-bound by construction).
    kernel_ms is the smaller of the two (still an upper bound, so `achieved`
    is never flattered); the median of per-launch event pairs (which adds ~2 us
    of event overhead) is reported beside them."""
    timed = span_ms / steps
    b2b = _per_launch_ms(fn, launches, dev, host_us=60.0)
    med = _median_launch_ms(fn, launches, dev)
    which = 'timed-region span' if timed <= b2b else 'back-to-back span'
    return min(timed, b2b), dict(
        kernel_ms_method=f'min(HIP event span around the {steps}-step timed region / steps, {launches} back-to-back '
                         f'launches in one event span / count) = {which}; launch stream; includes the inter-launch '
                         'dispatch gap',
        kernel_ms_timed_region=timed, kernel_ms_back_to_back=b2b, kernel_ms_event_pair_median=med)


def _traffic(kernel, workload, units, world):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/traffic.json, written by scripts/prof_summary.py from separate
    FETCH_SIZE and WRITE_SIZE passes: bytes = (2 x FETCH_SIZE + WRITE_SIZE) x
    1024, the gfx950 correction of MI355X_MICROARCH.md section HBM).  Only a
    record of the same workload, per-launch units (envs or samples) and world
    size counts; otherwise None (no PMC pass of this configuration)."""
    path = os.path.join(ROOT, 'profiles', 'traffic.json')
    try:
        with open(path) as f:
            rec = json.load(f).get(f'{kernel}@{workload}')
    except (OSError, ValueError):
        return None
    if not rec or rec.get('units') != units or rec.get('world', 1) != world:
        return None
    return rec.get('hbm_bytes_per_launch')


def bench_pointmaze(args, world, rank, dev):
    from ogbench_amd.sharding import shard

    total = args.num_envs
    base, n = shard(total, world, rank)
    ring = args.ring
    env, actions = _maze_job(total, base, n, ring, dev)
    views = list(actions.unbind(0))  # the ring's [n, 2] rows, indexed without a tensor op

    def step(i):
        env.step(views[i % ring])

    for i in range(args.warmup):
        step(i)
    span = []
    dt = _timed(step, args.steps, world, dev, span)
    value = total * args.steps / dt
    ms_per_step = dt / args.steps * 1e3

    # kernel duration for the roofline (the timed region's device span)
    kern_ms, kern_info = _launch_ms(span[0], args.steps, step, max(1000, min(args.steps, 2000)), dev)
    alg_bytes = 87 * n  # 87 B per env-step
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9

    extra = {'host_us_per_step': _host_us_per_call(step, 200, dev)}
    if args.no_extras:
        return _finish_pointmaze(args, world, rank, total, n, value, ms_per_step, kern_ms, alg_bytes, achieved,
                                 extra, env, kern_info)
    extra['eval_allgather'] = _eval_allgather(env, world, dev)
    env.reset(seed=0, options=dict(task_id=(torch.arange(base, base + n, dtype=torch.int32, device=dev) % 5) + 1))
    # K fused steps per launch (K = 1 and K = 100)
    K = 100
    fused_actions = actions[:K].contiguous()
    out = None

    def fused(i):
        nonlocal out
        out = env.rollout(fused_actions, out)

    fused(0)
    reps = max(1, args.steps // K)
    fdt = _timed(fused, reps, world, dev)
    extra[f'fused_k{K}_steps_per_s'] = total * K * reps / fdt
    fk_ms = _median_launch_ms(fused, 20, dev)
    fused_bytes = (8 + 16 + 4 + 3) * n * K + (16 + 16 + 4 + 4 + 16 + 4 + 4) * n
    extra[f'fused_k{K}_kernel_ms'] = fk_ms
    extra[f'fused_k{K}_achieved_GBs'] = fused_bytes / (fk_ms * 1e-3) / 1e9
    if world > 1:
        # weak scaling beside the strong-scaling value: 65,536 envs per GPU
        wn = 65536
        wenv, wact = _maze_job(wn * world, rank * wn, wn, ring, dev)
        for i in range(args.warmup):
            wenv.step(wact[i % ring])
        wdt = _timed(lambda i: wenv.step(wact[i % ring]), args.steps, world, dev)
        extra['weak_envs_per_gpu'] = wn
        extra['weak_total_envs'] = wn * world
        extra['weak_env_steps_per_s'] = wn * world * args.steps / wdt
        wenv.close()
    return _finish_pointmaze(args, world, rank, total, n, value, ms_per_step, kern_ms, alg_bytes, achieved, extra,
                             env, kern_info)


def _maze_job(total, base, n, ring, dev, maze='large'):
    """This rank's block [base, base+n) of a `total`-env pointmaze job: the
    handle at its global env_base, reset with the shared seed 0 and task i%5+1
    (global i), and its slice of the global action ring (seed 1, generated in
    8192-env blocks so that a rank never holds the whole ring)."""
    import ogbench_amd

    env = ogbench_amd.make(f'pointmaze-{maze}-v0', num_envs=n, device=dev, auto_reset=True, env_base=base)
    if 'OGBX_EPW' in os.environ:  # A/B knob: envs per 64-lane wave (results do not depend on it)
        from ogbench_amd import _lib
        _lib.check(env._L.ogbx_maze_set_envs_per_wave(env._h, int(os.environ['OGBX_EPW'])))
    task = (torch.arange(base, base + n, dtype=torch.int32, device=dev) % 5) + 1
    env.reset(seed=0, options=dict(task_id=task))
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    acts = torch.empty(ring, n, 2, device=dev, dtype=torch.float32)
    chunk = 8192
    for c0 in range(0, total, chunk):
        c1 = min(total, c0 + chunk)
        blk = torch.rand(ring, c1 - c0, 2, device=dev, generator=gen, dtype=torch.float32) * 2 - 1
        lo, hi = max(c0, base), min(c1, base + n)
        if lo < hi:
            acts[:, lo - base:hi - base] = blk[:, lo - c0:hi - c0]
    return env, acts


def _eval_allgather(env, world, dev, steps=1000):
    """Untimed: the eval success reduction of SURVEY section 8e.  Every env
    runs one episode of its task (i%5+1, global i) driven by the on-device
    point expert (BFS oracle subgoal + N(0, 0.2) noise, generate_locomaze.py:
    147-166); per-task {success, episodes} counters accumulate on the device
    over `steps` steps (1000 = the TimeLimit, so every env finishes its
    episode) and are all-gathered over the process group (RCCL over xGMI at
    N>1)."""
    from ogbench_amd.evaluation import accumulate, env_task_ids, gather_counters, summarize

    n, base = env.num_envs, env.env_base
    env.reset(seed=0, options=dict(task_id=(torch.arange(base, base + n, dtype=torch.int32, device=dev) % 5) + 1))
    counters = torch.zeros(env.num_tasks, 2, dtype=torch.int64, device=dev)
    remaining = torch.ones((n,), dtype=torch.int32, device=dev)
    tid = env_task_ids(env)
    act = None
    for i in range(steps):
        act = env.expert_action(noise=0.2, seed=0, out=act)
        _, _, term, trunc, info = env.step(act)
        accumulate(counters, info['success'].view(torch.uint8), term.view(torch.uint8), trunc.view(torch.uint8),
                   tid, remaining)
    _barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    total, per_rank = gather_counters(counters)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3
    m = summarize(total, env.task_infos)
    res = dict(episodes=int(total[:, 1].sum()), ranks=int(per_rank.shape[0]), policy='expert (noise 0.2)',
               overall_success=m.get('evaluation/overall_success'), allgather_ms=ms,
               per_task={k.split('/')[1]: v for k, v in m.items() if k != 'evaluation/overall_success'})
    if world > 1:
        # the C-ABI communicator (a second RCCL communicator per rank) has no
        # multi-GPU run on record yet: opt-in, so that an untried path cannot
        # stall the scaling run
        if os.environ.get('OGBX_BENCH_CABI_COMM') == '1':
            res.update(_cabi_allgather_check(counters, per_rank, world, dev))
        else:
            res['cabi_allgather'] = 'not run (set OGBX_BENCH_CABI_COMM=1)'
    return res


def _cabi_allgather_check(counters, per_rank, world, dev):
    """The same all-gather through the C-ABI communicator (ogbx_comm_* over
    RCCL, the path a non-Python host binds): must equal torch.distributed's.
    Reported, never fatal."""
    import torch.distributed as dist

    from ogbench_amd.evaluation import RcclComm, comm_unique_id

    try:
        if dist.get_backend() != 'nccl':
            return {'cabi_allgather': 'skipped (gloo rehearsal: RCCL needs one GPU per rank)'}
        uid = torch.zeros(128, dtype=torch.uint8, device=dev)
        if dist.get_rank() == 0:
            uid.copy_(torch.frombuffer(bytearray(comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        comm = RcclComm(world, dist.get_rank(), dev, bytes(uid.cpu().numpy().tobytes()))
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = comm.allgather(counters)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) * 1e3
        ok = bool(torch.equal(out.to(per_rank.device), per_rank))
        comm.close()
        return {'cabi_allgather_ms': ms, 'cabi_allgather_matches': ok}
    except Exception as e:  # pragma: no cover - reported, not fatal
        return {'cabi_allgather_error': repr(e)[:200]}


def _finish_pointmaze(args, world, rank, total, n, value, ms_per_step, kern_ms, alg_bytes, achieved, extra, env,
                      kern_info):
    result = dict(
        # BASELINE.json's metric at the default N = 65,536; a --num-envs run names its own N
        metric=f'env steps/sec at N={total} parallel envs, pointmaze-large, 1/2/4/8 MI355X',
        value=value,
        unit='env_steps/s',
        n_gpus=world,
        steps=args.steps,
        warmup=args.warmup,
        ms_per_step=ms_per_step,
        higher_is_better=True,
        scaling='strong',
        vs_baseline=None,
        dtype='f64',
        data='synthetic (uniform [-1,1] float32 actions, Philox reset noise; no dataset)',
        config=dict(
            workload='pointmaze-large-navigate-v0',
            total_envs=total,
            num_envs_per_gpu=n,
            auto_reset=True,
            task_id='i%5+1',
            seed=0,
            parallelism=f'env-shard x{world} (contiguous blocks, global env_base)',
        ),
        roofline=dict(
            # one wave's fp64 contact chain sets the launch time,
            # not HBM: achieved/peak are still the HBM figures of 87 B/env-step
            bound='latency',
            kernel='maze_step_kernel',
            achieved=achieved,
            peak=HBM_PEAK_GBS,
            unit='GB/s',
            frac=achieved / HBM_PEAK_GBS,
            traffic=_traffic('maze_step_kernel', 'pointmaze', n, world),
            kernel_ms=kern_ms,
            **kern_info,
            alg_bytes_per_launch=alg_bytes,
        ),
        extra=extra,
    )
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline_pointmaze(n, args)
    env.close()
    return result


def cpu_baseline_pointmaze(n, args):
    """The oracle C restatement (kind 'port'), OpenMP over envs, bounded sample."""
    from oracle import locomaze as orc

    threads = int(os.environ.get('OMP_NUM_THREADS', '16'))
    threads = max(1, min(threads, os.cpu_count() or 1))
    rng = np.random.RandomState(0)
    tid = (np.arange(n) % 5 + 1).astype(np.int32)
    st = orc.reset('large', tid, rng.uniform(-1, 1, (n, 4)))
    steps, t0 = 0, time.perf_counter()
    budget = args.cpu_seconds
    while time.perf_counter() - t0 < budget:
        a = rng.uniform(-1, 1, (1, n, 2)).astype(np.float32)
        orc.step('large', st, a, auto_reset=1, key=(0, 0), nthreads=threads)
        steps += 1
    dt = time.perf_counter() - t0
    return dict(
        value=n * steps / dt,
        unit='env_steps/s',
        cores=threads,
        kind='port',
        sample=f'{steps} steps x {n} envs of pointmaze-large with auto-reset ({dt:.1f} s)',
    )


def bench_pointmaze_n1(args, world, rank, dev):
    """pointmaze-medium-navigate-v0 with ONE env (BASELINE configs[0]; SURVEY 8d
    row 1: plumbing).  A step = one Gymnasium-surface ``env.step(action)`` of
    the single env through the C-ABI (one launch), actions U[-1,1]^2 float32
    from torch.Generator(seed=0) resident on the device, task 1 for every
    episode (same-step auto-reset keeps the stored task; TimeLimit 1000).  The number is
    launch-latency bound by construction (one env); ``cpu_baseline`` is the
    oracle C restatement stepping the same single env on 1 core (the
    reference MuJoCo step cannot run here: MuJoCo is absent)."""
    import ogbench_amd

    env = ogbench_amd.make('pointmaze-medium-v0', num_envs=1, device=dev, auto_reset=True)
    env.reset(seed=rank, options=dict(task_id=1))
    ring = 1000
    gen = torch.Generator(device='cpu').manual_seed(0)
    actions = (torch.rand(ring, 1, 2, generator=gen) * 2 - 1).float().to(dev)

    def step(i):
        env.step(actions[i % ring])

    for i in range(args.warmup):
        step(i)
    span = []
    dt = _timed(step, args.steps, world, dev, span)
    kern_ms, kern_info = _launch_ms(span[0], args.steps, step, 1000, dev)
    result = dict(
        metric='env steps/sec, pointmaze-medium-navigate-v0, N=1 env (Gymnasium surface)',
        value=args.steps * world / dt, unit='env_steps/s', n_gpus=world, steps=args.steps, warmup=args.warmup,
        ms_per_step=dt / args.steps * 1e3, higher_is_better=True, scaling='weak', vs_baseline=None, dtype='f64',
        data='synthetic (U[-1,1]^2 float32 actions, torch.Generator seed 0; Philox reset noise)',
        config=dict(workload='pointmaze-medium-navigate-v0 N=1', num_envs_per_gpu=1, auto_reset=True,
                    parallelism=f'replica x{world}'),
        roofline=dict(bound='latency', kernel='maze_step_kernel', achieved=87 / (kern_ms * 1e-3) / 1e9,
                      peak=HBM_PEAK_GBS, unit='GB/s', frac=87 / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                      traffic=None, kernel_ms=kern_ms, **kern_info, alg_bytes_per_launch=87),
        extra={},
    )
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline_pointmaze_n1(args)
    env.close()
    return result


def cpu_baseline_pointmaze_n1(args):
    """The oracle C restatement stepping one pointmaze-medium env per call
    (kind 'port', 1 core), as a Gymnasium loop would; auto-reset with Philox."""
    from oracle import locomaze as orc

    rng = np.random.RandomState(0)
    st = orc.reset('medium', np.array([1], np.int32), orc.reset_draws(1, 0))
    key = orc.philox_key(0, orc.TAG_MAZE_RESET)
    acts = rng.uniform(-1, 1, (1000, 1, 1, 2)).astype(np.float32)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < min(args.cpu_seconds, 5.0):
        for i in range(1000):
            orc.step('medium', st, acts[i], auto_reset=1, key=key, nthreads=1)
        steps += 1000
    dt = time.perf_counter() - t0
    return dict(value=steps / dt, unit='env_steps/s', cores=1, kind='port',
                sample=f'{steps} single-env steps of pointmaze-medium through the ctypes oracle ({dt:.1f} s)')


def bench_gcsample(args, world, rank, dev):
    """humanoidmaze-large-navigate-v0 offline replay: 1M-row buffer in HBM
    (500 trajectories x 2000 rows, obs 69 f32, act 21 f32), GCIQL humanoid
    config (discount 0.995), batch 1024.  A step = one GCDataset.sample(1024)
    (one fused launch).  Extra: 256 batches fused per launch."""
    from ogbench_amd.datasets import Dataset, GCDataset

    n_traj, L = 500, 2000
    R = n_traj * L
    g = torch.Generator(device=dev)
    g.manual_seed(3 + rank)
    term = torch.zeros(R, device=dev)
    term[L - 1 :: L] = 1
    data = dict(
        observations=torch.randn(R, 69, device=dev, generator=g),
        actions=torch.rand(R, 21, device=dev, generator=g) * 2 - 1,
        terminals=torch.clamp(term + torch.cat([term[1:], torch.ones(1, device=dev)]), max=1.0),
        valids=1.0 - term,
    )
    cfg = dict(discount=0.995, value_p_curgoal=0.2, value_p_trajgoal=0.5, value_p_randomgoal=0.3,
               value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=1.0, actor_p_randomgoal=0.0,
               actor_geom_sample=False, gc_negative=True, p_aug=0.0, frame_stack=None)
    if 'OGBX_GC_LOOKAHEAD' in os.environ:  # A/B knob (the sampler's lookahead config key)
        cfg['lookahead'] = os.environ['OGBX_GC_LOOKAHEAD'] != '0'
    gc = GCDataset(Dataset(data, device=dev), cfg, seed=rank)
    gc_kernel = 'gc_ahead_kernel<true>' if gc._lookahead else 'gc_sample_kernel'  # the launch of a steady call
    B = 1024
    batch = gc.sample(B)

    def step(i):
        # refill the previous batch in place (stream ordered; no per-call allocation)
        gc.sample(B, out=batch)

    def step_fresh(i):
        gc.sample(B)

    for i in range(args.warmup):
        step(i)
    span = []
    dt = _timed(step, args.steps, world, dev, span)
    value = B * args.steps * world / dt
    kern_ms, kern_info = _launch_ms(span[0], args.steps, step, 1000, dev)
    per_sample = 2424  # algorithmic bytes per sample (humanoid layout)
    achieved = per_sample * B / (kern_ms * 1e-3) / 1e9
    NB = 256

    def fused(i):
        gc.sample(B, num_batches=NB)

    extra = {'host_us_per_call': _host_us_per_call(step, 200, dev)}
    if not args.no_extras:
        fdt0 = _timed(step_fresh, args.steps, world, dev)
        extra['fresh_alloc_samples_per_s'] = B * args.steps * world / fdt0
        fused(0)
        reps = max(1, args.steps // 32)
        fdt = _timed(fused, reps, world, dev)
        fk_ms = _per_launch_ms(fused, 5, dev)
        extra.update(fused_256x1024_samples_per_s=B * NB * reps * world / fdt, fused_256x1024_kernel_ms=fk_ms,
                     fused_256x1024_achieved_GBs=per_sample * B * NB / (fk_ms * 1e-3) / 1e9)
    result = dict(
        metric='GCDataset.sample samples/sec, humanoidmaze-large-navigate-v0 1M-row buffer, batch 1024',
        value=value, unit='samples/s', n_gpus=world, steps=args.steps, warmup=args.warmup,
        ms_per_step=dt / args.steps * 1e3, higher_is_better=True, scaling='weak', vs_baseline=None,
        dtype='f32', data='synthetic (N(0,1) obs, U[-1,1] actions; 500 x 2000-row trajectories)',
        config=dict(workload='humanoidmaze-large-navigate-v0 offline replay', rows=R, batch=B,
                    agent_config='gciql humanoid (discount 0.995)', parallelism=f'replica x{world}'),
        # B = 1024 is a chain of HBM round trips (index loads, then rows), DESIGN 4.4
        roofline=dict(bound='latency', kernel=gc_kernel, achieved=achieved, peak=HBM_PEAK_GBS, unit='GB/s',
                      frac=achieved / HBM_PEAK_GBS, traffic=_traffic(gc_kernel, 'gcsample', B, world),
                      kernel_ms=kern_ms, **kern_info, alg_bytes_per_launch=per_sample * B),
        extra=extra,
    )
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline_gc(data, cfg, B, args)
    return result


def bench_hgcsample(args, world, rank, dev):
    """HGCDataset.sample(1024) on the same 1M-row humanoid buffer with the HIQL
    humanoidmaze config (discount 0.995, subgoal_steps 100; impls/hyperparameters.sh).
    A step = one sample(1024) refilling the previous batch (one fused launch)."""
    from ogbench_amd.datasets import Dataset, HGCDataset

    n_traj, L = 500, 2000
    R = n_traj * L
    g = torch.Generator(device=dev)
    g.manual_seed(3 + rank)
    term = torch.zeros(R, device=dev)
    term[L - 1 :: L] = 1
    data = dict(
        observations=torch.randn(R, 69, device=dev, generator=g),
        actions=torch.rand(R, 21, device=dev, generator=g) * 2 - 1,
        terminals=torch.clamp(term + torch.cat([term[1:], torch.ones(1, device=dev)]), max=1.0),
        valids=1.0 - term,
    )
    cfg = dict(discount=0.995, value_p_curgoal=0.2, value_p_trajgoal=0.5, value_p_randomgoal=0.3,
               value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=1.0, actor_p_randomgoal=0.0,
               actor_geom_sample=False, gc_negative=True, p_aug=0.0, frame_stack=None, subgoal_steps=100)
    if 'OGBX_GC_LOOKAHEAD' in os.environ:  # A/B knob (the sampler's lookahead config key)
        cfg['lookahead'] = os.environ['OGBX_GC_LOOKAHEAD'] != '0'
    hgc = HGCDataset(Dataset(data, device=dev), cfg, seed=rank)
    hgc_kernel = 'hgc_ahead_kernel<true>' if hgc._lookahead else 'hgc_sample_kernel'  # the launch of a steady call
    B = 1024
    batch = hgc.sample(B)

    def step(i):
        hgc.sample(B, out=batch)

    for i in range(args.warmup):
        step(i)
    span = []
    dt = _timed(step, args.steps, world, dev, span)
    kern_ms, kern_info = _launch_ms(span[0], args.steps, step, 1000, dev)
    # 12 gathered 276-B observation rows + actions 84 + terminals/valids 8,
    # read and written, + valid_idxs/traj_end lookups 16 + 9 x 8-B scalars written
    per_sample = 2 * (12 * 276 + 84 + 8) + 16 + 72
    achieved = per_sample * B / (kern_ms * 1e-3) / 1e9
    extra = {'host_us_per_call': _host_us_per_call(step, 200, dev)}
    if not args.no_extras:
        NB = 128
        big = hgc.sample(B, num_batches=NB)

        def fused(i):
            hgc.sample(B, num_batches=NB, out=big)

        reps = max(1, args.steps // 32)
        fdt = _timed(fused, reps, world, dev)
        fk_ms = _per_launch_ms(fused, 5, dev)
        extra.update(fused_128x1024_samples_per_s=B * NB * reps * world / fdt, fused_128x1024_kernel_ms=fk_ms,
                     fused_128x1024_achieved_GBs=per_sample * B * NB / (fk_ms * 1e-3) / 1e9)
    result = dict(
        metric='HGCDataset.sample samples/sec, humanoidmaze-large-navigate-v0 1M-row buffer, batch 1024',
        value=B * args.steps * world / dt, unit='samples/s', n_gpus=world, steps=args.steps, warmup=args.warmup,
        ms_per_step=dt / args.steps * 1e3, higher_is_better=True, scaling='weak', vs_baseline=None,
        dtype='f32', data='synthetic (N(0,1) obs, U[-1,1] actions; 500 x 2000-row trajectories)',
        config=dict(workload='humanoidmaze-large-navigate-v0 offline replay (HIQL sampler)', rows=R, batch=B,
                    agent_config='hiql humanoid (discount 0.995, subgoal_steps 100)',
                    parallelism=f'replica x{world}'),
        roofline=dict(bound='latency', kernel=hgc_kernel, achieved=achieved, peak=HBM_PEAK_GBS,
                      unit='GB/s', frac=achieved / HBM_PEAK_GBS,
                      traffic=_traffic(hgc_kernel, 'hgcsample', B, world),
                      kernel_ms=kern_ms, **kern_info, alg_bytes_per_launch=per_sample * B),
        extra=extra,
    )
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline_hgc(data, cfg, B, args)
    return result


def cpu_baseline_hgc(data, cfg, B, args):
    """The NumPy oracle restatement of HGCDataset.sample (kind 'port', 1 core)."""
    from oracle import gcdataset_np as orc

    host = {k: v.cpu().numpy() for k, v in data.items()}
    prep = orc.prepare(host)
    nvalid = len(prep['valid'])
    rng = np.random.RandomState(0)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        d = dict(pick=rng.randint(nvalid, size=B))
        for p, geom in (('v_', True), ('a_', False)):
            d[p + 'pick'] = rng.randint(nvalid, size=B)
            if geom:
                d[p + 'geom'] = rng.geometric(1 - cfg['discount'], size=B)
            else:
                d[p + 'dist'] = rng.rand(B)
            d[p + 'u_traj'] = rng.rand(B)
            d[p + 'u_cur'] = rng.rand(B)
        orc.hgc_sample(host, cfg, d, prep=prep)
        n += 1
    dt = time.perf_counter() - t0
    return dict(value=n * B / dt, unit='samples/s', cores=1, kind='port',
                sample=f'{n} batches of {B} on the 1M-row humanoid buffer ({dt:.1f} s; valid_idxs and '
                       'terminal_locs computed once before the loop, as HGCDataset.__post_init__ does)')


def cpu_baseline_gc(data, cfg, B, args):
    """The NumPy oracle restatement of GCDataset.sample (kind 'port', 1 core),
    with np.random draws in the reference's call order, on the same buffer."""
    from oracle import gcdataset_np as orc

    host = {k: v.cpu().numpy() for k, v in data.items()}
    prep = orc.prepare(host)
    valid = prep['valid']
    rng = np.random.RandomState(0)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        d = dict(pick=rng.randint(len(valid), size=B))
        for p, geom in (('v_', True), ('a_', False)):
            d[p + 'pick'] = rng.randint(len(valid), size=B)
            if geom:
                d[p + 'geom'] = rng.geometric(1 - cfg['discount'], size=B)
            else:
                d[p + 'dist'] = rng.rand(B)
            d[p + 'u_traj'] = rng.rand(B)
            d[p + 'u_cur'] = rng.rand(B)
        orc.sample(host, cfg, d, prep=prep)
        n += 1
    dt = time.perf_counter() - t0
    return dict(value=n * B / dt, unit='samples/s', cores=1, kind='port',
                sample=f'{n} batches of {B} on the 1M-row humanoid buffer ({dt:.1f} s; valid_idxs and '
                       'terminal_locs computed once before the loop, as GCDataset.__post_init__ does)')


def bench_powder(args, world, rank, dev, level='easy'):
    """powderworld-{level}-v0, 64x64 worlds, N=4096 envs per GPU (SURVEY.md section 8 row b;
    medium/hard: section 8f).  A step = one env.step of all envs (one step-kernel launch;
    medium/hard: the render-only kernel then the full-rule kernel),
    uniformly random valid actions for the current stage, task i%5+1, same-step auto-reset
    (medium/hard: the auto-reset replays the task's goal in the same launch, as the
    reference's reset does)."""
    import ogbench_amd

    n = 4096 if args.num_envs == 65536 else args.num_envs
    size = 64
    ne = {'easy': 2, 'medium': 5, 'hard': 8}[level]
    full = ne != 2
    # medium/hard: a single step is two launches, the render-only kernel for envs
    # whose step runs no forward and the full-rule kernel for the rest
    kern = 'pwf_light_step_kernel+pwf_step_kernel' if full else 'pw_step_kernel'
    env = ogbench_amd.make(f'powderworld-{level}-v0', num_envs=n, device=dev, world_size=size, auto_reset=True)
    task = (torch.arange(n, dtype=torch.int32, device=dev) % 5) + 1
    env.reset(seed=rank, options=dict(task_id=task))
    gen = torch.Generator(device=dev)
    gen.manual_seed(5 + 1000 * rank)
    ring = 3 * 32
    xy = env._xy_action_size
    hi = torch.tensor([ne if i % 3 == 0 else xy for i in range(ring)], device=dev).view(ring, 1)
    actions = (torch.rand(ring, n, device=dev, generator=gen) * hi).to(torch.int32)

    def step(i):
        env.step(actions[i % ring])

    for i in range(args.warmup):
        step(i)
    steps = args.steps - args.steps % 3 if args.steps >= 3 else args.steps
    span = []
    dt = _timed(step, steps, world, dev, span)
    value = n * steps * world / dt
    # device time per step of the timed region itself (one HIP event pair on
    # the launch stream around it): the world's contents, and with them the
    # forward's cost, drift over an episode, so a separate window would price
    # different states; the mean also spans whole 3-step action cycles
    kern_ms = span[0] / steps
    # algorithmic bytes per env-step.  easy: obs write H*W*6, world read H*W,
    # world write H*W on one step in three, action 4, reward 4, flags 3, ctrl
    # 16.  medium/hard (render-cache design), per cell and 3-step
    # action cycle: the forward step reads the 10-byte state (id, momentum,
    # velocity) and the goal id, writes the state, the 3-byte render cache
    # and the 6-byte obs (30 B); each of the two render-only steps reads the
    # cache and writes the obs (9 B) -- 48 B per 3 steps = 16 B/cell/step.
    if full:
        per_step = size * size * 16 + 27
    else:
        per_step = size * size * (6 + 1 + 1 / 3) + 27
    achieved = per_step * n / (kern_ms * 1e-3) / 1e9
    extra = {}
    K = 48
    fk_actions = actions[:K].contiguous()
    out = None

    def fused(i):
        nonlocal out
        out = env.rollout(fk_actions, out=out)

    if full and not args.no_extras:
        extra.update(_powder_phases(env, step, steps, dev))
    if not args.no_extras:
        fused(0)
        reps = max(1, steps // K)
        fdt = _timed(fused, reps, world, dev)
        fk_ms = _per_launch_ms(fused, 3, dev)
        extra.update(fused_k48_steps_per_s=n * K * reps * world / fdt, fused_k48_kernel_ms=fk_ms,
                     fused_k48_achieved_GBs=per_step * n * K / (fk_ms * 1e-3) / 1e9)
    result = dict(
        metric=f'env steps/sec, powderworld-{level}-v0 64x64, N={n} parallel envs per GPU',
        value=value, unit='env_steps/s', n_gpus=world, steps=steps, warmup=args.warmup,
        ms_per_step=dt / steps * 1e3, higher_is_better=True, scaling='weak', vs_baseline=None,
        dtype='f32+u8' if full else 'u8',
        data='synthetic (uniform valid Discrete actions per stage; Philox resets' + (' and rand fields)' if full else ')'),
        config=dict(workload=f'powderworld-{level}-v0 world_size=64', num_envs_per_gpu=n, auto_reset=True,
                    parallelism=f'env-shard x{world}'),
        # easy: HBM-bound; medium/hard: VALU issue-bound (one world per CU,
        # its 16 waves keep the SIMDs issuing)
        roofline=dict(bound='issue' if full else 'hbm', kernel=kern, achieved=achieved, peak=HBM_PEAK_GBS,
                      unit='GB/s', frac=achieved / HBM_PEAK_GBS, traffic=_traffic(kern, args.workload, n, world),
                      kernel_ms=kern_ms, alg_bytes_per_launch=per_step * n,
                      alg_bytes_basis=(f'{per_step:.0f} B/env-step: 16 B/cell/step over the 3-step action cycle '
                                       '(forward step: 10-B state read + write, goal id, 3-B render cache and 6-B '
                                       'obs written; render-only steps: cache read, obs written; DESIGN 4.3)'
                                       if full else
                                       f'{per_step:.0f} B/env-step for the 1-byte cell state; supersedes SURVEY 8d\'s '
                                       '55,979 B, which prices a 10-byte state whose extra channels the easy rules '
                                       'never make non-zero (DESIGN 4.2)')),
        extra=extra,
    )
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline_powder_full(ne, size, args) if full else cpu_baseline_powder(size, args)
    env.close()
    return result


def cpu_baseline_powder(size, args):
    """The NumPy oracle (kind 'port', 1 core): one env at a time, random valid actions."""
    from oracle import powder_np as orc
    from ogbench_amd.powder_tasks import easy_task_sequences

    rng = np.random.RandomState(0)
    o = orc.Env(size)
    ids, grav, didg = o.blank()
    for e, x, y in easy_task_sequences()[0]:
        ids, grav, didg = orc.paint(*orc.forward(ids, grav, didg), orc.EASY_ELEMS[e], x, y)
    o.reset(ids, 0, 3, 3)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        a = rng.randint(0, 2 if o.stage == 0 else o.xy)
        _, _, succ = o.step(int(a))
        n += 1
        if succ or n % 500 == 0:
            o.reset(ids, rng.randint(2), rng.randint(o.xy), rng.randint(o.xy))
    dt = time.perf_counter() - t0
    return dict(value=n / dt, unit='env_steps/s', cores=1, kind='port',
                sample=f'{n} single-env steps of powderworld-easy {size}x{size} ({dt:.1f} s)')


def _powder_phases(env, step, start, dev):
    """Medium/hard: the steady-state step and the synchronized auto-reset step
    priced apart (device time on the launch stream).  Every env starts its
    episode together, so all of them auto-reset (goal replay) in the same step
    every max_episode_steps steps (envs that reach their goal earlier reset on
    their own, rarely under random actions).  Steady state: the mean of a
    window of whole 3-step action cycles that contains no synchronized reset;
    reset step: the one step in which the synchronized reset happens."""
    el = int(env._scalar_view('elapsed')[0])  # (state_dict would mark the render cache stale)
    T = env.max_episode_steps
    left = T - el  # the step with index start + left - 1 is the synchronized reset
    i = start
    stream = torch.cuda.current_stream(dev)
    ev = lambda: torch.cuda.Event(enable_timing=True)
    win = min(300, left - 1) // 3 * 3
    out = {}
    if win >= 3:
        a, b = ev(), ev()
        torch.cuda.synchronize(dev)
        a.record(stream)
        for _ in range(win):
            step(i)
            i += 1
        b.record(stream)
        torch.cuda.synchronize(dev)
        out['steady_state_ms_per_step'] = a.elapsed_time(b) / win
        out['steady_state_window_steps'] = win
    while i < start + left - 1:  # up to the step before the reset
        step(i)
        i += 1
    a, b = ev(), ev()
    torch.cuda.synchronize(dev)
    a.record(stream)
    step(i)
    b.record(stream)
    torch.cuda.synchronize(dev)
    out['sync_reset_step_ms'] = a.elapsed_time(b)
    out['sync_reset_envs'] = int((env._scalar_view('elapsed') == 0).sum())
    out['sync_reset_every_steps'] = T
    return out


def cpu_baseline_powder_full(ne, size, args):
    """The NumPy oracle of the full rule set (kind 'port', 1 core): one env at a
    time, random valid actions, rand fields from np.random as the reference."""
    from oracle import powder_full_np as orc
    from ogbench_amd.powder_tasks import task_sequences

    rng = np.random.RandomState(0)
    o = orc.Env(ne, size)
    H = size

    def rand():
        return [rng.rand(H, H).astype(np.float32) for _ in range(3)]

    seq = task_sequences(ne)[0]
    goal = o.replay(seq[:8], [rand() for _ in seq[:8]])[0, 0].astype(np.uint8)  # a short goal replay
    o.reset(goal, 0, 3, 3, rand())
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        a = rng.randint(0, ne if o.stage == 0 else o.xy)
        o.step(int(a), rand())
        o.errors()
        n += 1
    dt = time.perf_counter() - t0
    return dict(value=n / dt, unit='env_steps/s', cores=1, kind='port',
                sample=f'{n} single-env steps of powderworld-{"medium" if ne == 5 else "hard"} {size}x{size} '
                       f'({dt:.1f} s; goal replays excluded)')


ANT_BYTES = 15 * 8 + 14 * 8  # one body state row (qpos 15 + qvel 14, f64)


def bench_antmaze(args, world, rank, dev):
    """antmaze-large-navigate-v0 wrapper (BASELINE configs[4]: N = 131,072 over
    8 GPUs = 16,384 envs per rank, weak scaling): one step = ogbx_antmaze_step
    over this rank's envs consuming a caller-supplied post-physics body state
    (a ring of 8 synthetic snapshots standing in for the out-of-scope ant
    dynamics), same-step auto-reset with Philox reset bodies, task i%5+1 of
    the global env index.  Algorithmic bytes per env-step: post-physics row
    read 232 + body state write 232 + ob write 232 + goal 16 + elapsed 8 +
    reward/flags 7 = 727 B (SURVEY 8d prices the same contract at 759 B with
    the physics engine's action read, which the wrapper does not touch)."""
    import ogbench_amd
    from ogbench_amd.evaluation import accumulate, env_task_ids, gather_counters, summarize

    n = args.num_envs if args.num_envs != 65536 else 16384
    base = rank * n
    env = ogbench_amd.MazeEnv('ant', 'large', num_envs=n, device=dev, auto_reset=True, env_base=base)
    tid = (torch.arange(base, base + n, dtype=torch.int32, device=dev) % 5) + 1
    obs0, info = env.reset(seed=0, options=dict(task_id=tid))
    R = 8
    gen = torch.Generator(device=dev)
    gen.manual_seed(1 + rank)
    goal = env.cur_goal_xy  # info['goal'] is the 29-d goal observation
    start = obs0[:, :2].clone()
    ring_q = torch.randn(R, n, 15, device=dev, dtype=torch.float64, generator=gen)
    ring_v = torch.randn(R, n, 14, device=dev, dtype=torch.float64, generator=gen)
    # snapshots walk part of the way to the goal: some envs reach it (success,
    # termination, auto-reset), the rest run to the TimeLimit
    frac = (torch.rand(n, 1, device=dev, dtype=torch.float64, generator=gen) * 1.25).clamp(max=1.0)
    for k in range(R):
        ring_q[k, :, :2] = start + (goal - start) * frac * (k + 1) / R

    # the engine's output buffers: R fixed (qpos, qvel) pairs, reused every R
    # steps as a physics engine reuses its state buffers (wrap_step's cached path)
    rq, rv = list(ring_q.unbind(0)), list(ring_v.unbind(0))

    def step(i):
        env.wrap_step(rq[i % R], rv[i % R])

    for i in range(args.warmup):
        step(i)
    span = []
    dt = _timed(step, args.steps, world, dev, span)
    value = n * world * args.steps / dt
    kern_ms, kern_info = _launch_ms(span[0], args.steps, step, max(1000, min(args.steps, 2000)), dev)
    per = 3 * ANT_BYTES + 16 + 8 + 7
    achieved = per * n / (kern_ms * 1e-3) / 1e9
    extra = {}
    if not args.no_extras:
        # untimed eval reduction over the wrapper's flags
        counters = torch.zeros(env.num_tasks, 2, dtype=torch.int64, device=dev)
        remaining = torch.ones(n, dtype=torch.int32, device=dev)
        ids = env_task_ids(env)
        for i in range(1000):
            _, _, te, tr, inf = env.wrap_step(rq[i % R], rv[i % R])
            accumulate(counters, inf['success'].view(torch.uint8), te.view(torch.uint8), tr.view(torch.uint8), ids,
                       remaining)
        total, per_rank = gather_counters(counters)
        m = summarize(total, env.task_infos)
        extra['eval_allgather'] = dict(episodes=int(total[:, 1].sum()), ranks=int(per_rank.shape[0]),
                                       policy='synthetic post-physics ring',
                                       overall_success=m.get('evaluation/overall_success'))
    result = dict(
        metric='antmaze wrapper env steps/sec, antmaze-large-navigate-v0, 16384 envs per GPU',
        value=value, unit='env_steps/s', n_gpus=world, steps=args.steps, warmup=args.warmup,
        ms_per_step=dt / args.steps * 1e3, higher_is_better=True, scaling='weak', vs_baseline=None, dtype='f64',
        data='synthetic post-physics ant states (ring of 8 snapshots; ant dynamics out of scope), Philox resets',
        config=dict(workload='antmaze-large-navigate-v0 wrapper', num_envs_per_gpu=n, total_envs=n * world,
                    auto_reset=True, task_id='i%5+1', parallelism=f'env-shard x{world} (global env_base)'),
        roofline=dict(bound='hbm', kernel='ant_step_kernel', achieved=achieved, peak=HBM_PEAK_GBS, unit='GB/s',
                      frac=achieved / HBM_PEAK_GBS, traffic=_traffic('ant_step_kernel', 'antmaze', n, world),
                      kernel_ms=kern_ms, **kern_info, alg_bytes_per_launch=per * n),
        extra=extra,
    )
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline_antmaze(n, args)
    env.close()
    return result


def cpu_baseline_antmaze(n, args):
    """oracle/antmaze_np.py (NumPy, 1 core) on the same workload shape."""
    from oracle import antmaze_np as am

    rng = np.random.RandomState(0)
    task = np.arange(n) % 5 + 1
    b = am.Batch(task, rng.uniform(-1, 1, (n, 4)), np.concatenate(
        [rng.uniform(-0.1, 0.1, (n, 15)), rng.standard_normal((n, 14))], 1))
    R = 8
    qs = [rng.standard_normal((n, 15)) for _ in range(R)]
    vs = [rng.standard_normal((n, 14)) for _ in range(R)]
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < min(args.cpu_seconds, 10.0):
        b.step(qs[steps % R], vs[steps % R], auto_reset=True, rng=rng)
        steps += 1
    dt = time.perf_counter() - t0
    return dict(value=n * steps / dt, unit='env_steps/s', cores=1, kind='port',
                sample=f'{steps} steps x {n} envs of the wrapper with auto-reset ({dt:.1f} s)')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--warmup', type=int, default=100)
    ap.add_argument('--workload', default='pointmaze',
                    choices=['pointmaze', 'pointmaze-medium-n1', 'powder', 'powder-medium', 'powder-hard', 'gcsample',
                             'hgcsample', 'antmaze'])
    ap.add_argument('--num-envs', type=int, default=65536)
    ap.add_argument('--ring', type=int, default=128)
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-extras', action='store_true', help='only the timed single-step workload (profiling runs)')
    ap.add_argument('--dist-backend', default='nccl', choices=['nccl', 'gloo'],
                    help="'gloo' rehearses the multi-rank path with ranks sharing GPUs")
    args = ap.parse_args()
    # before any HIP call: refuse a mismatched layout, or start the N ranks
    if _check_world(args.gpus, args.dist_backend) == 'self-launch':
        rc, _ = _self_launch(args.gpus, sys.argv[1:])
        sys.exit(rc)
    world, rank, local = _dist_init(args.dist_backend)
    dev = torch.device('cuda', local)
    sys.path.insert(0, ROOT)
    fn = dict(pointmaze=bench_pointmaze, powder=bench_powder, **{'pointmaze-medium-n1': bench_pointmaze_n1},
              gcsample=bench_gcsample, hgcsample=bench_hgcsample, antmaze=bench_antmaze,
              **{'powder-medium': lambda *a: bench_powder(*a, level='medium'),
                 'powder-hard': lambda *a: bench_powder(*a, level='hard')})[args.workload]
    result = fn(args, world, rank, dev)
    result['ranks_seen'] = _ranks_seen(world, dev)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == '__main__':
    main()
