"""Pre-tuned solutions for the library GEMMs of the training step (PyTorch TunableOp over hipBLASLt / rocBLAS).

The projection GEMMs of the encoder (245760 x 512 x 512 at 256 videos, forward / dgrad / split-K wgrad) are
~60% of the step.  hipBLASLt's default heuristic picks a tile that reaches 121-137 TF/s on them; an exhaustive
search over the hipBLASLt and rocBLAS solutions for the exact shapes finds 138-145 TF/s (fp32 MFMA peak ~157;
tools/tunable_probe.py).  tools/tune_gemms.py runs the search once for the bench workload and writes
`tuning/gemm_gfx950.csv` (op, shape, solution id, time).  `enable()` loads that table with tuning off: a GEMM
whose shape is in the table calls the recorded solution, any other shape keeps the default heuristic.  The
table is keyed by PyTorch / ROCm / hipBLASLt / rocBLAS versions and the gfx arch; TunableOp ignores it when
they differ.  Same arithmetic (fp32 inputs, fp32 accumulate); only the tiling (summation order) changes.
"""
import os
import shutil
import tempfile

import torch

TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "gemm_gfx950.csv")


def enable(table: str = TABLE, tag: str = "") -> bool:
    """Use the tuned GEMM table (if present) for every later GEMM of this process; returns whether it was found.
    TunableOp reads its file on first use and rewrites it at exit, so it gets a private copy."""
    if not os.path.exists(table):
        return False
    import torch.cuda.tunable as tun
    work = os.path.join(tempfile.gettempdir(), f"pdvc_gemm_table_{os.getpid()}{tag}.csv")
    shutil.copyfile(table, work)
    tun.set_filename(work)
    tun.tuning_enable(False)
    tun.enable(True)
    return True


def disable() -> None:
    import torch.cuda.tunable as tun
    tun.enable(False)
