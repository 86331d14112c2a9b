"""Achievable HBM bandwidth probes (pdp_stream_copy variants, 8 GiB device
copy, (read + write) bytes / time):  python tools/copy_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pipelinedp_amd import native
    torch.cuda.init()
    for variant, grid in ((0, 8192), (1, 8192), (0, 2048), (1, 2048), (1, 32768), (0, 8192)):
        os.environ["PDP_COPY_VARIANT"] = str(variant)
        os.environ["PDP_COPY_GRID"] = str(grid)
        print(f"variant {variant} grid {grid}: {bench.copy_peak_gbs(torch, native.lib())} GB/s", flush=True)


if __name__ == "__main__":
    main()
