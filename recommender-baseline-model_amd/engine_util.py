"""Helpers shared by the SAS and BERT engines."""
import numpy as np
import torch


def compute_dtype(args):
    """``args.rs_dtype``: 'fp32' (default: the reference's precision, parity mode) or 'bf16'."""
    name = str(getattr(args, "rs_dtype", "fp32") or "fp32").lower()
    if name in ("fp32", "float32", "f32"):
        return torch.float32
    if name in ("bf16", "bfloat16"):
        return torch.bfloat16
    raise ValueError(f"rs_dtype must be fp32 or bf16, got {name!r}")


def as_ids(x, device):
    """numpy / list / tensor -> contiguous int64 device tensor (the reference's
    ``torch.LongTensor(x).to(device)``, BS/models/sas_model/sas.py:60,93-94)."""
    if isinstance(x, torch.Tensor):
        t = x.to(device=device, dtype=torch.int64, non_blocking=True)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(x, dtype=np.int64))).to(device, non_blocking=True)
    return t.contiguous()


def require_cuda(device):
    if torch.device(device).type != "cuda":
        raise RuntimeError(
            "rbm_amd runs the training hot path only through its HIP kernels (librecsys_hip.so); "
            "set args.device='cuda' (there is no CPU fallback)")


def site_salt(base, site):
    """Distinct 64-bit dropout salt per (model instance, dropout site)."""
    return (int(base) * 0x100000001B3 + 0x9E3779B97F4A7C15 * (site + 1)) & 0xFFFFFFFFFFFFFFFF


class Workspace:
    """Per-shape scratch buffers reused across steps (the C ABI allocates nothing)."""

    def __init__(self, device):
        self.device = device
        self.bufs = {}

    def get(self, name, shape, dtype):
        shape = tuple(int(s) for s in shape)
        t = self.bufs.get(name)
        if t is None or t.dtype != dtype or tuple(t.shape) != shape:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self.bufs[name] = t
        return t


# Events created while a stream is capturing a HIP graph are kept alive until that capture has ended
# (FusedTrainStep._capture_graphs releases them after instantiation): a per-step event dropped mid-capture -- the
# next unrolled step replacing it, a local going out of scope -- is otherwise destroyed while the capture still tracks
# it as a dependency source.
_CAPTURE_EVENTS = []


def capture_event():
    """torch.cuda.Event() for a fork / join inside a step; held until the end of the capture when one is running."""
    ev = torch.cuda.Event()
    if torch.cuda.is_current_stream_capturing():
        _CAPTURE_EVENTS.append(ev)
    return ev


def release_capture_events():
    _CAPTURE_EVENTS.clear()
