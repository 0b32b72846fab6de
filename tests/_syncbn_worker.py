"""One rank of the synchronised-BatchNorm GPU test (tests/test_gpu_dp.py::
test_sync_batchnorm_two_ranks_equal_global_batch): a fresh child process per rank, gloo,
both ranks on cuda:0.  PGUNet{stage} on this rank's contiguous shard of the global batch,
every BatchNorm synchronised (ugpg.dist.enable_sync_batchnorm), weighted BCE, backward, the
trainer's gradient all-reduce; dumps logits, averaged gradients and BN buffers."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ug-pg-unet_amd")]


def main(outdir, stage, B, res, math="x6"):
    import torch
    import torch.distributed as dist
    import torch.nn as nn
    from oracle import detgen as G
    from tests._parity import det_state
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    import ugpg
    from ugpg import ops
    from ugpg.dist import allreduce_gradients, enable_sync_batchnorm, shard
    ops.set_conv_math(math)
    enable_sync_batchnorm(True)
    stage, B, res = int(stage), int(B), int(res)
    state = det_state(stage, 3, 1)
    x = G.randn(1, (B, 3, res, res), "x")
    t = G.bernoulli(2, (B, 1, res, res), 0.5, "t")
    m = getattr(ugpg, f"PGUNet{stage}")(3, 1)
    m.load_state_dict(state)
    m = m.to("cuda").train()
    xs, ts = shard(x, rank, 2).cuda(), shard(t, rank, 2).cuda()
    out = m(xs)
    crit = nn.BCEWithLogitsLoss(pos_weight=torch.tensor([5.0], device="cuda"), reduction="none")
    final, _ = ugpg.UncertaintyGuidedLoss("cuda").apply_uncertainty_weighted_loss(crit, out, ts)
    final.backward()
    params = list(m.parameters())
    scale = allreduce_gradients(params)
    torch.cuda.synchronize()
    names = [k for k, _ in m.named_parameters()]
    torch.save({"logits": out.detach().cpu(),
                "grads": {k: (p.grad * scale).cpu() for k, p in zip(names, params)},
                "bufs": {k: v.detach().cpu() for k, v in m.state_dict().items()
                         if k.endswith(("running_mean", "running_var", "num_batches_tracked"))}},
               os.path.join(outdir, f"rank{rank}.pt"))
    enable_sync_batchnorm(False)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(*sys.argv[1:])
