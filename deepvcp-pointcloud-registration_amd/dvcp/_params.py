"""Packing of nn.Module parameters into the flat fp32 buffers the HIP kernels read.

The packed buffer is cached on the owning module and rebuilt only when a parameter or BN
buffer changes (tracked by tensor version counters and storage pointers), so inference runs
pack once.  Packing is plain tensor concatenation on the parameters' device.
"""
import torch


def _key(tensors):
    return tuple((t.data_ptr(), t._version, t.device) for t in tensors)


def cached_pack(module, tag, tensors, build):
    cache = module.__dict__.setdefault("_dvcp_pack", {})
    key = _key(tensors)
    hit = cache.get(tag)
    if hit is not None and hit[0] == key:
        return hit[1]
    with torch.no_grad():
        buf = build().detach().float().contiguous()
    cache[tag] = (key, buf)
    return buf


def bn_affine(bn):
    """Eval-mode BatchNorm as y = x * scale + shift (torch's CPU inference kernel form)."""
    scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    shift = bn.bias - bn.running_mean * scale
    return scale, shift


def linear_pack(*linears):
    """[W (out x in) row-major, bias] per layer, back to back."""
    parts = []
    for lin in linears:
        parts += [lin.weight.reshape(-1), lin.bias.reshape(-1)]
    return torch.cat(parts)


def linear_tensors(*linears):
    out = []
    for lin in linears:
        out += [lin.weight, lin.bias]
    return out
