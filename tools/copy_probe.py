"""Achievable HBM bandwidth probes (pdp_stream_copy variants over an 8 GiB
buffer; copies count read + write bytes, the read-only / write-only variants
the bytes they move):  python tools/copy_probe.py  -> one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = {0: "copy plain 4-deep", 1: "copy nt/nt 8-deep", 2: "copy nt loads, default stores",
         3: "copy default/default 8-deep", 4: "copy default loads, nt stores", 5: "read only nt",
         6: "read only default", 7: "write only nt", 8: "write only default"}


def probe(torch, lib, variant, grid, nbytes=8 << 30, iters=5):
    os.environ["PDP_COPY_VARIANT"] = str(variant)
    os.environ["PDP_COPY_GRID"] = str(grid)
    src = torch.empty(nbytes // 8, dtype=torch.int64, device="cuda")
    dst = torch.empty_like(src)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        if lib.pdp_stream_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), nbytes, stream):
            raise RuntimeError("pdp_stream_copy failed")

    run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        run()
    b.record()
    torch.cuda.synchronize()
    moved = nbytes * (2 if variant <= 4 else 1)
    return round(moved * iters / (a.elapsed_time(b) * 1e-3) / 1e9, 1)


def main():
    import torch
    from pipelinedp_amd import native
    torch.cuda.init()
    lib = native.lib()
    out = {}
    for variant in range(9):
        for grid in (2048, 8192, 32768):
            out[f"{variant}:{grid}"] = (NAMES[variant], probe(torch, lib, variant, grid))
            print(variant, grid, out[f"{variant}:{grid}"], flush=True)
    print(json.dumps({"copy_probe_GBs": out}), flush=True)


if __name__ == "__main__":
    main()
