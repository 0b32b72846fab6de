"""Test helpers that make out-of-bounds writes and reads of unwritten memory visible
(VERDICT r4 "next" item 1).

guarded(): a tensor placed in the middle of a larger device buffer whose guard bands hold
a NaN canary pattern; `check()` asserts the bands are bit-for-bit intact, so a kernel that
writes past either end of its operand fails the test that launched it instead of silently
corrupting a neighbouring allocation.

poison_cache(): NaN-fill the memory the caching allocator hands out next (its freed large
block and a few hundred small-pool segments), so a kernel that reads memory nobody wrote
in this step sees NaN instead of whatever a previous kernel or process left there.
"""
import math

import torch

# quiet-NaN payloads, recognisable in a dump
CANARY32 = 0x7FBADBAD
CANARY16 = 0x7FBD


class Guarded:
    __slots__ = ("buf", "t", "pad", "n", "_iv")

    def __init__(self, shape, dev, dtype=torch.float32, pad=16384, fill=None):
        n = math.prod(shape)
        self.pad, self.n = pad, n
        self.buf = torch.empty(pad + n + pad, dtype=dtype, device=dev)
        if dtype in (torch.float32, torch.int32):
            self._iv = self.buf.view(torch.int32)
            self._iv.fill_(CANARY32)
        elif dtype in (torch.bfloat16, torch.float16, torch.int16):
            self._iv = self.buf.view(torch.int16)
            self._iv.fill_(CANARY16)
        else:
            self._iv = self.buf.view(torch.uint8)
            self._iv.fill_(0xA5)
        self.t = self.buf[pad:pad + n].view(shape)
        if fill is not None:
            self.t.copy_(fill)

    def check(self, name="buffer"):
        want = self._iv[:self.pad].clone()
        want.fill_(CANARY32 if self._iv.dtype == torch.int32 else
                   CANARY16 if self._iv.dtype == torch.int16 else 0xA5)
        for side, band in (("before", self._iv[:self.pad]), ("after", self._iv[self.pad + self.n:])):
            bad = (band != want).nonzero()
            assert bad.numel() == 0, (
                f"{name}: {bad.numel()} guard elements overwritten {side} the tensor "
                f"(first at offset {int(bad[0]) - (self.pad if side == 'before' else 0)} "
                f"{'from its start' if side == 'before' else 'past its end'})")


def guarded(shape, dev, dtype=torch.float32, fill=None, pad=16384):
    return Guarded(tuple(shape), dev, dtype, pad, fill)


def poison_cache(dev, value=float("nan")):
    """Fill what the caching allocator will hand out next with `value`: release the cache,
    then allocate, fill and free one large block (later large allocations split it) and 256
    small ones (the small pool's 2 MiB segments).  NaN alone is not a complete poison --
    fmaxf-based ReLU and max-pool drop it -- so tests run twice with two different fills
    and require bit-identical results."""
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(dev)
    big = torch.empty(int(min(free * 0.5, 16e9)) // 4, device=dev).fill_(value)
    small = [torch.empty(1 << 17, device=dev).fill_(value) for _ in range(256)]
    del big, small
    torch.cuda.synchronize(dev)
