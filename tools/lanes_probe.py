"""Probe: does splitting a rank's shard into L concurrent lanes (one itsd_unet handle + HIP stream each)
raise the step rate at small N, where every launch is latency-bound?

Times W graph-replayed steps of (a) one handle over the whole batch of N and (b) L handles over N/L each,
their sampler runs issued on L different caller streams so the graphs can overlap on the hardware queues.
Also checks that each lane's images match the same candidates run alone in a batch of N/L (bit for bit: the
trajectory is a function of (seed, global index) and the lane's kernels are those of batch N/L).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import itsd  # noqa: E402,F401
import itsd.runtime as rt  # noqa: E402
from itsd.arch import ARCH_A  # noqa: E402
from itsd.schedule import make_schedule  # noqa: E402
from itsd.weights import synthetic_state_dict  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, nargs="+", default=[16, 32, 64])
    p.add_argument("--lanes", type=int, nargs="+", default=[2])
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--reps", type=int, default=3)
    args = p.parse_args()
    a = ARCH_A
    sd = synthetic_state_dict(a, 0)
    s = make_schedule(1e-4, 0.02, a.T)
    sched = (s.coeff1_f32, s.coeff2_f32, s.sqrt_var_f32, 0.0)
    handles = {}

    def handle(key, cap):
        if key not in handles:
            h = rt.NativeUNet(a, sd, cap, rt.PREC_BF16, 0)
            h.set_schedule(*sched)
            handles[key] = h
        return handles[key]

    per = 3 * 32 * 32
    T0 = a.T - 1
    for n in args.n:
        x0 = torch.randn(n, 3, 32, 32, device="cuda")
        h = handle(("whole", n), n)

        def run_whole(steps):
            x = x0.clone()
            h.run(x, T0, T0 - steps + 1, 7, noise_offset=0, clip=False, sync=False)
            return [x]

        for L in args.lanes:
            if n % L:
                continue
            m = n // L
            hs = [handle(("lane", m, i), m) for i in range(L)]
            ss = [torch.cuda.Stream() for _ in range(L)]

            def run_lanes(steps):
                xs = [x0[i * m:(i + 1) * m].clone() for i in range(L)]
                torch.cuda.synchronize()
                for i in range(L):
                    with torch.cuda.stream(ss[i]):
                        hs[i].run(xs[i], T0, T0 - steps + 1, 7, noise_offset=i * m * per, clip=False, sync=False)
                return xs

            # correctness: lanes vs each lane alone (serial)
            xs = run_lanes(args.steps)
            torch.cuda.synchronize()
            ok = True
            for i in range(L):
                xi = x0[i * m:(i + 1) * m].clone()
                hs[i].run(xi, T0, T0 - args.steps + 1, 7, noise_offset=i * m * per, clip=False, sync=True)
                ok &= bool(torch.equal(xi, xs[i]))
            xw = run_whole(args.steps)[0]
            torch.cuda.synchronize()
            rel = ((torch.cat(xs) - xw).norm() / xw.norm()).item()
            res = {}
            for name, fn in (("whole", run_whole), ("lanes", run_lanes)):
                fn(5)
                torch.cuda.synchronize()
                best = 1e9
                for _ in range(args.reps):
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    fn(args.steps)
                    torch.cuda.synchronize()
                    best = min(best, time.perf_counter() - t)
                res[name] = best / args.steps * 1e3
            print(f"N={n:4d} L={L}: whole {res['whole']:.4f} ms/step  lanes {res['lanes']:.4f} ms/step  "
                  f"ratio {res['lanes'] / res['whole']:.3f}  lane==alone {ok}  rel-L2 lanes vs whole {rel:.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
