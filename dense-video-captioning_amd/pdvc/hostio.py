"""Host -> device transfers that do not stall the GPU.

`torch.tensor(list, device=cuda)` and `.to(cuda)` of a pageable CPU tensor are blocking copies (PyTorch's
memcpy-and-sync path): each one drains the stream, so a step with a dozen of them runs the host and the
GPU in lock-step.  Here small host arrays go through pinned memory with non_blocking=True (the caching host
allocator keeps the pinned block alive until the copy has run), and several index arrays share one copy.
"""
import numpy as np
import torch


def to_device(x, device, dtype=None):
    """list / ndarray / CPU tensor -> device tensor, asynchronously."""
    t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
    if dtype is not None:
        t = t.to(dtype)
    if t.device.type != "cpu" or torch.device(device).type == "cpu":
        return t.to(device)
    if torch.cuda.is_current_stream_capturing():
        # a copy node would re-read this host buffer at every replay, after it has been freed
        raise RuntimeError("host->device copy inside a graph capture: cache the device tensor before capturing")
    return t.pin_memory().to(device, non_blocking=True)


def pack_to_device(arrays, device, dtype=torch.int64):
    """Several 1-D host arrays -> list of device tensors from ONE asynchronous copy."""
    arrays = [np.asarray(a).reshape(-1) for a in arrays]
    sizes = [a.size for a in arrays]
    flat = np.concatenate(arrays) if arrays else np.zeros(0)
    t = to_device(flat, device, dtype)
    return list(torch.split(t, sizes))


_CONST = {}


def const(key, fn, device):
    """A per-device cached constant tensor (built once by fn() on the host)."""
    k = (key, str(device))
    t = _CONST.get(k)
    if t is None:
        t = _CONST[k] = to_device(fn(), device)
    return t
