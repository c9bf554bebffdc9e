#!/usr/bin/env python3
"""Achievable HBM bandwidth on this GPU for the access mixes of the pipeline: pure write (fill), pure read
(sum), copy (1 read : 1 write) and 1 read : 2.5 write (the rate dematcher's mix).  torch kernels, timed with
events; prints one JSON line."""
import json

import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3


def main():
    n = 2_400_000_000 // 4
    a = torch.empty(n, dtype=torch.float32, device="cuda")
    b = torch.empty(n, dtype=torch.float32, device="cuda")
    small = torch.empty(n * 2 // 5, dtype=torch.float32, device="cuda")
    res = {}
    t = timed(lambda: a.fill_(1.0))
    res["write_TBps"] = round(a.numel() * 4 / t / 1e12, 2)
    t = timed(lambda: a.sum())
    res["read_TBps"] = round(a.numel() * 4 / t / 1e12, 2)
    t = timed(lambda: b.copy_(a))
    res["copy_TBps"] = round(2 * a.numel() * 4 / t / 1e12, 2)
    # 1 : 2.5 mix: read `small` (0.4 n) and write a 2.5x larger view by broadcasting
    v = a.view(-1, 5)[:, :2]
    w = small.view(-1, 2)
    t = timed(lambda: a.view(-1, 5).copy_(w.repeat(1, 3)[:, :5]))
    res["note"] = "fill/sum/copy are torch kernels; the mixed probe includes a repeat temporary"
    print(json.dumps(res))


if __name__ == "__main__":
    main()
