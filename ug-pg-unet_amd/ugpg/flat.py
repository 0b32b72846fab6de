"""One contiguous fp32 buffer per model for its parameters (HBM layout).

Parameters stay ordinary ``nn.Parameter`` objects with the reference's
state_dict keys, but their storage is re-pointed into one flat buffer in
``module.parameters()`` order.  Gradients come back in a buffer with the same
layout (functional.py), so RMSprop is one kernel launch and the data-parallel
gradient exchange is one RCCL all-reduce over a single tensor.
"""
from __future__ import annotations

import torch


def contiguous_run(tensors):
    """If `tensors` are back-to-back views of one storage (in order), return
    (base_tensor_1d, start_offset, total_numel); else None."""
    if not tensors or any(t is None for t in tensors):
        return None
    st = tensors[0].untyped_storage()
    ptr0 = st.data_ptr()
    off = tensors[0].storage_offset()
    start = off
    for t in tensors:
        if t.untyped_storage().data_ptr() != ptr0 or t.storage_offset() != off or not t.is_contiguous():
            return None
        off += t.numel()
    if tensors[0].dtype != torch.float32:
        return None
    base = torch.empty(0, dtype=torch.float32, device=tensors[0].device).set_(
        st, start, (off - start,), (1,))
    return base, start, off - start


def ensure_flat(module: torch.nn.Module) -> None:
    params = [p for p in module.parameters()]
    if not params or not params[0].is_cuda:
        return
    if contiguous_run(params) is not None:
        return
    dev = params[0].device
    total = sum(p.numel() for p in params)
    flat = torch.empty(total, dtype=torch.float32, device=dev)
    off = 0
    cur = torch.cuda.current_stream(dev)
    with torch.no_grad():
        for p in params:
            n = p.numel()
            flat[off:off + n].copy_(p.data.reshape(-1))
            # the old storage dies here while the copy may still be pending on the current
            # stream: if it was allocated on another stream, its block must not go back to
            # that stream's pool before the copy has read it
            p.data.record_stream(cur)
            p.data = flat[off:off + n].view_as(p)
            off += n
