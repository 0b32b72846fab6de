"""libugpg's RCCL communicator (C-ABI ugpg_comm_*) on one GPU: a
single-rank communicator's all-reduce (sum/avg/max) and broadcast are identities, stream
ordered, in place, for every dtype the trainer exchanges.  Multi-rank exchange needs one GPU
per rank (RCCL refuses two ranks on one device), so the N-rank numerics are covered by the
torch.distributed path (tests/test_gpu_dp.py, gloo) that shares the reducer code."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_single_rank_communicator(dev):
    from ugpg.dist import Communicator
    c = Communicator(rank=0, world_size=1, device=torch.cuda.current_device())
    try:
        for dt in (torch.float32, torch.bfloat16, torch.float64, torch.int64):
            x = (torch.arange(1000, device=dev) % 97).to(dt)
            want = x.clone()
            for op in ("sum", "avg", "max"):
                if dt == torch.int64 and op == "avg":
                    continue
                c.all_reduce(x, op)
                torch.cuda.synchronize()
                assert torch.equal(x, want), (dt, op)
            c.broadcast(x, 0)
            torch.cuda.synchronize()
            assert torch.equal(x, want)
        with pytest.raises(RuntimeError):
            c.all_reduce(torch.zeros(4))  # host tensor
    finally:
        c.close()
