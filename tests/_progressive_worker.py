"""One rank of the 2-process progressive-driver GPU test (tests/test_gpu_progressive.py):
a fresh child process per rank (never exec'd from a GPU-initialised process), gloo,
both ranks on cuda:0.  Runs ugpg's UncertaintyGuidedProgressiveTrainer.train_progressive
(config 5, uncertainty_guided_trainer.py:316-398) on the G12 data exactly as a user would
under torchrun, recording for every stage: the stage model's state right after each
train_epoch (before the buffer broadcast that precedes validation) and the state of every
stage model when the next stage starts (after the stage-end broadcast)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ug-pg-unet_amd")]


def main(outdir):
    import torch
    import torch.distributed as dist
    from torch.utils.data import DataLoader, TensorDataset
    from oracle.make_goldens import G12, g12_data
    from tests._parity import det_state
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    import ugpg

    def snap(m):
        return {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}

    class Recording(ugpg.UncertaintyGuidedProgressiveTrainer):
        after_train, at_stage_end = [], {}

        def train_epoch(self, dataloader, stage):
            tup = super().train_epoch(dataloader, stage)
            self.after_train.append((stage, snap(self.models[stage])))
            return tup

        def transfer_weights(self, prev_stage, new_stage):
            self.at_stage_end[prev_stage] = snap(self.models[prev_stage])
            super().transfer_weights(prev_stage, new_stage)

    torch.manual_seed(0)
    tr = Recording(3, 1, device="cuda", uncertainty_alpha=1.0)
    for s in range(1, 5):
        tr.models[s].load_state_dict(det_state(s, 3, 1, seed=G12["w_seeds"][s]))
        tr.stage_configs[s]["lr"] = 0.0
        tr.stage_configs[s]["epochs_per_stage"] = G12["epochs"]
    tr.setup_optimizer(1)
    x, t, vx, vt = g12_data()
    bs = G12["bs"]
    tl = DataLoader(TensorDataset(x, t), batch_size=bs, shuffle=False)
    vl = DataLoader(TensorDataset(vx, vt), batch_size=bs, shuffle=False)
    save = os.path.join(outdir, f"ck_rank{rank}")
    tr.train_progressive(tl, vl, max_stages=4, save_dir=save)
    torch.cuda.synchronize()
    tr.at_stage_end[4] = snap(tr.models[4])
    torch.save({"history": tr.history, "after_train": tr.after_train,
                "at_stage_end": tr.at_stage_end,
                "ckpts": sorted(os.listdir(save))},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
