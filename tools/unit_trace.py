#!/usr/bin/env python3
"""Per-unit schedule of one render launch (debug build PTG_UNIT_TRACE=1):
where a frame or shard loses time to its grid end.

  make -C cpu-path-tracing_amd variant NAME=trace DEFS=-DPTG_UNIT_TRACE=1
  PTGPU_LIB=cpu-path-tracing_amd/build/libptgpu_trace.so \\
      python tools/unit_trace.py [--scene box] [--shards 8] [--rank 0]

Every unit (one wave) records its start and end (s_memrealtime, 100 MHz)
and hardware id.  Reported: the launch span, the busy fraction of the
device's wave slots over it (sum of unit durations / (span x slots)), the
number of units running over time (tenths of the span), unit durations by
position in the unit order (head / tail levels), and how the CUs' last ends
spread.  Prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-path-tracing_amd"))

import torch  # noqa: E402

import ptgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="box")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--shards", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--chunk", type=int, default=0)
    args = ap.parse_args()
    W, H, samps = args.width, args.height, args.spp // 4
    scn = ptgpu.make_scene(args.scene, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    lib = ptgpu.lib()
    p = ptgpu.make_params(W, H, samps, 2, ptgpu.DEFAULT_SEED, 1, args.rank, args.shards, args.chunk)
    rows = ptgpu.shard_rows(H, 1, args.shards)
    slab = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
    with ptgpu.Context(scn, cam, device=0) as ctx:
        info = ctx.launch_info(p)
        n = int(info["units"])
        buf = np.zeros(3 * n, dtype=np.uint64)
        ctx.render_device(slab, p)  # warm-up
        torch.cuda.synchronize()
        lib.ptg_unit_trace_(buf.ctypes.data_as(C.c_void_p), C.c_int(n))  # zero
        ctx.render_device(slab, p)
        torch.cuda.synchronize()
        lib.ptg_unit_trace_(buf.ctypes.data_as(C.c_void_p), C.c_int(n))
    t = buf.reshape(n, 3)
    ok = t[:, 1] > 0  # (padding units before a cooperative level never run)
    t0 = t[ok, 0].min()
    st = (t[:, 0].astype(np.int64) - int(t0)) / 100.0  # microseconds
    en = (t[:, 1].astype(np.int64) - int(t0)) / 100.0
    st, en = st[ok], en[ok]
    dur = en - st
    span = float(en.max())
    slots = int(torch.cuda.get_device_properties(0).multi_processor_count) * 32
    tenths = [int(((st <= span * (k + 0.5) / 10) & (en > span * (k + 0.5) / 10)).sum()) for k in range(10)]
    idx = np.nonzero(ok)[0]
    parts = {}
    for name, lo, hi in (("first_half", 0, n // 2), ("third_quarter", n // 2, 3 * n // 4),
                         ("last_quarter", 3 * n // 4, n - n // 32), ("last_32nd", n - n // 32, n)):
        m = (idx >= lo) & (idx < hi)
        if m.any():
            parts[name] = {"units": int(m.sum()), "mean_us": round(float(dur[m].mean()), 1),
                           "cv": round(float(dur[m].std() / max(dur[m].mean(), 1e-9)), 3)}
    hw = t[ok, 2]
    cu_key = (hw >> np.uint64(32)) * np.uint64(4096) + ((hw >> np.uint64(8)) & np.uint64(0xF)) \
        + ((hw >> np.uint64(13)) & np.uint64(0x7)) * np.uint64(16) + ((hw >> np.uint64(12)) & np.uint64(1)) * np.uint64(128)
    last = {}
    for k, e in zip(cu_key.tolist(), en.tolist()):
        last[k] = max(last.get(k, 0.0), e)
    le = np.array(sorted(last.values()))
    # the idle slot-time after the first CU runs out of work
    out = {"workload": f"{args.scene} {W}x{H} {args.spp}spp", "shard": f"{args.rank}/{args.shards}", "units": n,
           "span_ms": round(span / 1e3, 3), "slots": slots,
           "slot_busy_fraction": round(float(dur.sum() / (span * slots)), 4),
           "running_units_at_tenths": tenths, "durations": parts,
           "cu_last_end_ms": {"n_cu": len(le), "min": round(float(le.min()) / 1e3, 3),
                              "p10": round(float(np.percentile(le, 10)) / 1e3, 3),
                              "median": round(float(np.median(le)) / 1e3, 3), "max": round(float(le.max()) / 1e3, 3)},
           "launch_info": info}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
