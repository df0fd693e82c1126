"""Build nn.Module trees whose ``state_dict`` keys equal the reference checkpoint keys.

The modules only hold parameters (PyTorch is plumbing here: device memory, ``.cuda()``,
``load_state_dict``); all compute goes through ``libttship.so``.
"""

import torch
from torch import nn

BUFFER_KINDS = {"bn_mean", "bn_var", "count", "buffer"}


class Container(nn.Module):
    """Plain parameter holder (one level of a dotted state_dict key)."""

    def forward(self, *args, **kwargs):  # pragma: no cover - never called
        raise RuntimeError("parameter container; use the model's inference()")


def child(root: nn.Module, path):
    m = root
    for p in path:
        if p not in m._modules:
            m.add_module(p, Container())
        m = m._modules[p]
    return m


def populate(root: nn.Module, spec, skip_prefixes=()):
    """Register every (name, shape, kind) of ``spec`` under ``root`` (zeros; loaded later)."""
    for name, shape, kind in spec:
        if any(name.startswith(p) for p in skip_prefixes):
            continue
        *path, leaf = name.split(".")
        m = child(root, path)
        if kind == "count":
            m.register_buffer(leaf, torch.zeros(shape, dtype=torch.long))
        elif kind in BUFFER_KINDS:
            m.register_buffer(leaf, torch.zeros(shape, dtype=torch.float32))
        else:
            setattr(m, leaf, nn.Parameter(torch.zeros(shape, dtype=torch.float32), requires_grad=False))
    return root


def host_tensors(module: nn.Module, skip_prefixes=(), skip_kinds=("num_batches_tracked",)):
    """state_dict as contiguous fp32 numpy arrays (what the C ABI's set_tensor takes)."""
    out = {}
    for k, v in module.state_dict().items():
        if any(k.startswith(p) for p in skip_prefixes) or k.split(".")[-1] in skip_kinds:
            continue
        out[k] = v.detach().to("cpu", torch.float32).contiguous().numpy()
    return out


_TOKENS = __import__("itertools").count(1)


def new_token() -> int:
    """Process-unique model identity for the engine's weight cache (never reused, unlike id())."""
    return next(_TOKENS)
