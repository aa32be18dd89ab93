"""Adam kernel over the cfg-2 live range (457.3M fp32 params): HIP-event time per launch and
HBM rate (28 B/param: read p, g, m, v; write p, m, v). usage: python tools/adam_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from savqa_amd import ops  # noqa: E402


def main():
    n = 457_300_000 // 64 * 64
    dev = torch.device("cuda", 0)
    p, g, m, v = (torch.rand(n, device=dev) for _ in range(4))
    for _ in range(3):
        ops.adam(p, g, m, v, n, 1e-4, 0.9, 0.999, 1e-8, 0.1, 0.001, 1.0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    it = 10
    for _ in range(it):
        ops.adam(p, g, m, v, n, 1e-4, 0.9, 0.999, 1e-8, 0.1, 0.001, 1.0)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(f"{os.environ.get('SAVQA_LIB', 'cur')}: {ms:.3f} ms  {28 * n / ms / 1e6:.0f} GB/s")


if __name__ == "__main__":
    main()
