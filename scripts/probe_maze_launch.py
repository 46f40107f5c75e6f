"""Diagnostic: per-launch time of the pointmaze kernels on warmed-up states
(300 random-action steps with auto-reset), median of HIP event pairs.

  * maze_step_kernel at N = 65,536 and N = 8,192 (the 8-GPU strong share) for
    several envs-per-wave settings;
  * point_physics_kernel on all envs, on the contact envs only (compacted)
    and on the free envs only: the fixed cost of a launch vs the contact chain.
Run with OGBX_LIB=... to probe a variant build."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ogbench_amd  # noqa: E402

dev = torch.device('cuda', 0)


def med_us(fn, reps=400):
    for _ in range(20):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    t = sorted(s.elapsed_time(e) for s, e in ev)
    return t[len(t) // 2] * 1e3


def warmed(n):
    env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=dev, auto_reset=True)
    env.reset(seed=0, options=dict(task_id=(torch.arange(n, device=dev, dtype=torch.int32) % 5) + 1))
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    acts = torch.rand(64, n, 2, device=dev, generator=g) * 2 - 1
    for i in range(300):
        env.step(acts[i % 64])
    return env, acts


for n, epws in ((65536, (64, 32, 16)), (8192, (64, 32, 16, 8))):
    env, acts = warmed(n)
    q0 = env.get_xy().clone()
    for epw in epws:
        env._L.ogbx_maze_set_envs_per_wave(env._h, epw)
        k = [0]

        def step():
            env.step(acts[k[0] % 64])
            k[0] += 1

        print(f'N={n:6d} epw={epw:2d}: step {med_us(step):7.2f} us', flush=True)
    env._L.ogbx_maze_set_envs_per_wave(env._h, 64)
    a = acts[0].contiguous()
    out, cf = env.physics(q0, a)
    c = cf.bool()
    qc, ac = q0[c].contiguous(), a[c].contiguous()
    qf, af = q0[~c].contiguous(), a[~c].contiguous()
    print(f'N={n:6d} physics all {med_us(lambda: env.physics(q0, a)):7.2f} us | contact-only ({int(c.sum())}) '
          f'{med_us(lambda: env.physics(qc, ac)):7.2f} us | free-only {med_us(lambda: env.physics(qf, af)):7.2f} us',
          flush=True)
    env.close()
