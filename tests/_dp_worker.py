"""One rank of the data-parallel GPU test (tests/test_gpu_dp.py): started as a fresh
child process per rank (never exec'd from a GPU-initialised process), gloo backend,
both ranks on cuda:0.  Runs ugpg's trainer exactly as a user would under torchrun:
constructor (replica broadcast), load_stage_weights (rank 1 loads DIFFERENT weights,
which the broadcast must overwrite), train_epoch on a global-batch DataLoader (each rank
keeps its shard), then dumps gradients, parameters, buffers and the epoch tuple."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ug-pg-unet_amd")]


def main(outdir, math="x6", exchange="fp32"):
    os.environ["UGPG_GRAD_BF16"] = "1" if exchange == "bf16" else "0"
    import torch
    import torch.distributed as dist
    from torch.utils.data import DataLoader, TensorDataset
    from oracle import detgen as G
    from oracle.make_goldens import G8 as c
    from tests._parity import det_state, perturbed_state
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    torch.manual_seed(1000 + rank)               # replicas start different on purpose
    import ugpg
    from ugpg import ops
    ops.set_conv_math(math)  # "bf16": config 3's arithmetic (exchange: fp32 default, bf16 opt-in)
    tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device="cuda", uncertainty_alpha=1.0)
    p0 = {k: v.detach().cpu().clone() for k, v in tr.models[3].state_dict().items()}
    stage = c["stage"]
    state = det_state(stage, 3, 1, seed=c["w_seed"])
    if rank != 0:
        state = perturbed_state(state, 77, 1e-2)
    ck = os.path.join(outdir, f"ck{rank}.pth")
    torch.save({"model_state_dict": state}, ck)
    tr.load_stage_weights(stage, ck)             # broadcast: rank 0's weights everywhere
    tr.models[stage - 1].load_state_dict(det_state(stage - 1, 3, 1, seed=c["prev_seed"]))
    tr.current_stage, tr.current_model = stage, tr.models[stage]
    tr.setup_optimizer(stage)
    x = G.randn(c["x_seed"], (c["B"], 3, c["res"], c["res"]), "x")
    t = G.bernoulli(c["t_seed"], (c["B"], 1, c["res"], c["res"]), 0.5, "t")
    tup = tr.train_epoch(DataLoader(TensorDataset(x, t), batch_size=c["B"]), stage)
    torch.cuda.synchronize()
    m = tr.models[stage]
    # this rank's own (pre-exchange) gradient: the same step on a fresh replica of the
    # initial weights, outside any data-parallel exchange
    local = {}
    if math == "bf16":
        import torch.nn as nn
        fresh = ugpg.PGUNet2(3, 1).to("cuda")
        fresh.load_state_dict(det_state(stage, 3, 1, seed=c["w_seed"]))
        fresh.train()
        per = c["B"] // 2
        xs = x[rank * per:(rank + 1) * per].cuda()
        ts = t[rank * per:(rank + 1) * per].cuda()
        u = tr.uncertainty_loss.generate_uncertainty_map(xs, tr.models[stage - 1], 32, 64)
        crit = nn.BCEWithLogitsLoss(pos_weight=torch.tensor([5.0], device="cuda"),
                                    reduction="none")
        f, _ = tr.uncertainty_loss.apply_uncertainty_weighted_loss(crit, fresh(xs), ts, u, 1.0)
        f.backward()
        torch.cuda.synchronize()
        local = {k: p.grad.detach().cpu() for k, p in fresh.named_parameters()}
    torch.save({"tuple": tup, "local": local,
                "grads": {k: p.grad.detach().cpu() for k, p in m.named_parameters()},
                "state": {k: v.detach().cpu() for k, v in m.state_dict().items()},
                "ctor_s3": p0,
                "ctor_s3_after": {k: v.detach().cpu() for k, v in tr.models[3].state_dict().items()}},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:4]))
