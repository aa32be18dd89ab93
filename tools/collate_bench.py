#!/usr/bin/env python
"""Batch collation, reference path vs device path.

reference : collate_fn restated (oracle/collate.py == onlyobj:341-445 / super_node:366-497,
            numpy on one host core) + the per-tensor `.cuda()` copies of main:260-316
            (pageable memory, as the reference's DataLoader has no pin_memory)
device    : collate.pack (host) + one pinned H2D copy + savqa_collate/_edges kernels.
Kernel time is HIP-event timed on the launch stream with the packed bytes already in
HBM; bytes = dense bytes written + packed bytes read. Prints one JSON line per workload.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle import collate as ocol  # noqa: E402  (reference leg only)
from savqa_amd import collate  # noqa: E402
from savqa_amd.data import synthetic_samples  # noqa: E402

HBM_PEAK = 8000.0  # GB/s, MI355X_MICROARCH.md


def wall(fn, reps, warm=1):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def run(name, data, relations, reps=5, kreps=50):
    ref_fn = ocol.collate_super_node if relations else ocol.collate_onlyobj
    dense = ref_fn(data)
    dense_bytes = sum(v.nbytes for v in dense.values())

    def ref_path():
        d = ref_fn(data)
        return {k: torch.from_numpy(v).cuda() for k, v in d.items()}
    t_ref_host = wall(lambda: ref_fn(data), reps)
    t_ref = wall(ref_path, reps)

    t_pack_fresh = wall(lambda: collate.pack(data, relations), reps)
    pk = collate.pack(data, relations).pin_memory()
    pinned = pk.staging
    t_pack = wall(lambda: collate.pack(data, relations, staging=pinned), reps)

    def dev_path():
        return collate.to_device(pk)
    t_dev = wall(dev_path, reps)
    ring = collate.StagingRing(2)
    t_ring = wall(lambda: ring.collate(data, relations), reps, warm=2)
    # kernels alone, packed bytes resident: the launches are captured once into a HIP
    # graph so the host's ctypes overhead does not leave the GPU idle between them
    db = collate.DeviceBatch(pk, torch.device("cuda", torch.cuda.current_device()),
                             pk.staging.cuda())
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        db.launch(side.cuda_stream)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            db.launch(side.cuda_stream)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(kreps):
        g.replay()
    e1.record(s)
    torch.cuda.synchronize()
    t_k = e0.elapsed_time(e1) / kreps * 1e-3
    moved = dense_bytes + pk.nbytes
    B = pk.B
    line = {"workload": name, "batch": B, "dense_MB": round(dense_bytes / 1e6, 2),
            "packed_MB": round(pk.nbytes / 1e6, 2),
            "reference_ms": {"host_collate": round(t_ref_host * 1e3, 3),
                             "collate_plus_cuda_copies": round(t_ref * 1e3, 3)},
            "device_ms": {"pack_reused_pinned": round(t_pack * 1e3, 3),
                          "pack_fresh_buffer": round(t_pack_fresh * 1e3, 3),
                          "staging_ring_end_to_end": round(t_ring * 1e3, 3),
                          "h2d_plus_kernels": round(t_dev * 1e3, 3),
                          "kernels_resident": round(t_k * 1e3, 4)},
            "samples_per_s": {"reference": round(B / t_ref, 1),
                              "device_staging_ring": round(B / t_ring, 1)},
            "roofline": {"bound": "hbm", "achieved": round(moved / t_k / 1e9, 1),
                         "peak": HBM_PEAK, "unit": "GB/s",
                         "frac": round(moved / t_k / 1e9 / HBM_PEAK, 3)}}
    print(json.dumps(line), flush=True)


def main():
    torch.set_num_threads(1)
    run("cfg2_onlyobj", synthetic_samples(256, seed=3), False)
    run("super_node_rel", synthetic_samples(4, relations=True, Nv=(36, 36), Lq=(14, 14),
                                            seed=4), True)


if __name__ == "__main__":
    main()
