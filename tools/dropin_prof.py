"""The drop-in operator (MultiScaleDeformableAttention.ms_deform_attn_backward) at PDVC's lifted encoder pyramid --
run under rocprofv3 --kernel-trace --stats to see which kernels its backward launches and what each costs.
    python tools/dropin_prof.py [--videos 256] [--reps 5]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dense-video-captioning_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import bench
    res = bench.dropin_msda(512, videos=a.videos, reps=a.reps)
    print(res)


if __name__ == "__main__":
    main()
