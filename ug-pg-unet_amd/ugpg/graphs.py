"""hipGraph capture of a whole training step (opt-in: ``trainer.enable_graphs()`` or
UGPG_GRAPHS=1; ``bench.py --graph``).

An eager step issues about 200 kernel launches from Python (5-7 ms of host time,
profiles/r6i_host_probe_*.txt); a captured step is replayed with one call.  The captured
kernels, their arguments and the buffers they use are fixed, so a replay computes exactly
what the eager step computes from the same state (tests/test_gpu_graphs.py).  Where the
host's issue time bounds the step -- small batches and images -- a replay runs 1.5x the
eager rate (bs2 x 64^2: 6.07 -> 3.90 ms; bs4 x 128^2: 6.15 -> 4.15 ms); at the benchmarked
bs16 x 256^2 the GPU bounds the step and the two are equal (profiles/r6l_graph_probe.txt).

What a capture bakes in is the caller's key: input shapes, hyperparameters, the
identities of modules and parameters, the versions of tensors the step reads but does not
write (the frozen previous stage).  A key not seen before runs eagerly once, then captures.
"""
from __future__ import annotations

import torch


class StepGraph:
    """One captured step ``fn(*inputs)``: static copies of the inputs (refreshed from the
    caller's tensors before every replay), the graph, and ``fn``'s output tensor (rewritten
    by every replay).  Capturing only records: the step runs at the first replay."""

    def __init__(self, key, fn, inputs):
        self.key = key
        self.inputs = [torch.empty_like(t) for t in inputs]
        for s, t in zip(self.inputs, inputs):
            s.copy_(t)
        dev = self.inputs[0].device
        self.graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            with torch.cuda.graph(self.graph, stream=side):
                self.out = fn(*self.inputs)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.replays = 0

    def replay(self, inputs):
        for s, t in zip(self.inputs, inputs):
            if s.data_ptr() != t.data_ptr():
                s.copy_(t)
        self.graph.replay()
        self.replays += 1
        return self.out
