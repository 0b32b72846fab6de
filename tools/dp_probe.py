"""Where does the 2-rank config-5 run (tests/test_gpu_progressive.py two-rank test) lose
run-to-run determinism?  (diagnostic)

Stage-2 trainer from the G12 weights, lr 0, the G12 images: three train epochs, printing
per batch this rank's LOCAL metrics (before the metrics all-reduce) and checksums of the
stage's logits and U map.  With lr 0 every epoch must repeat the first bit for bit.

    python tools/dp_probe.py single        # one process, batch size 1 (the ranks' shard size)
    python tools/dp_probe.py dp            # 2 ranks (gloo, both on cuda:0), global bs 2
    python tools/dp_probe.py rank          # (internal: one rank)
    python tools/dp_probe.py poison        # one process: each step first fills every free
                                           # block of the caching allocator with NaN
"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]


def poison_cache(dev):
    """Fill the caching allocator's free memory with NaN: release the cache, then allocate,
    NaN-fill and free one large block (the large pool's next allocations split it) and a
    few hundred small ones (the small pool's 2 MiB segments).  A kernel that reads memory
    nobody wrote in this step then sees NaN instead of yesterday's (deterministic) data."""
    import torch
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    big = torch.empty(int(min(free * 0.6, 24e9)) // 4, device=dev).fill_(float("nan"))
    small = [torch.empty(1 << 17, device=dev).fill_(float("nan")) for _ in range(256)]
    del big, small
    torch.cuda.synchronize()


def run(bs, tag, poison=False, stage=2, epochs=3):
    import torch
    from torch.utils.data import DataLoader, TensorDataset
    import ugpg
    from oracle.make_goldens import G12, g12_data
    from tests._parity import det_state

    class Probe(ugpg.UncertaintyGuidedProgressiveTrainer):
        def _forward_device(self, data, target, stage, mbuf):
            m = self.models[stage]
            psum = sum(float(p.detach().double().sum()) for p in m.parameters())
            out = super()._forward_device(data, target, stage, mbuf)
            with torch.no_grad():  # the same forward again (train-mode BN, no autograd)
                again = float(m(data).double().sum())
            self._probe = (float(out[0].detach().double().sum()),
                           float(out[1].double().sum()) if out[1] is not None else 0.0,
                           float(data.double().sum()), psum, again)
            return out

        def train_step(self, data, target, stage):
            if poison:
                poison_cache(data.device)
            return super().train_step(data, target, stage)

        def _reduce_metrics(self, mbuf, umap):
            v = mbuf.tolist()
            print(f"{tag} local {' '.join(f'{x:.9g}' for x in v[:7])} | logits {self._probe[0]:.9g} "
                  f"U {self._probe[1]:.9g} data {self._probe[2]:.9g} params {self._probe[3]:.12g} "
                  f"again {self._probe[4]:.9g}", flush=True)
            super()._reduce_metrics(mbuf, umap)

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    tr = Probe(3, 1, device=dev, uncertainty_alpha=1.0)
    for s in range(1, 5):
        tr.models[s].load_state_dict(det_state(s, 3, 1, seed=G12["w_seeds"][s]))
        tr.stage_configs[s]["lr"] = 0.0
    tr.current_stage, tr.current_model = stage, tr.models[stage]
    tr.setup_optimizer(stage)
    x, t, _, _ = g12_data()
    tl = DataLoader(TensorDataset(x, t), batch_size=bs, shuffle=False)
    for ep in range(epochs):
        tup = tr.train_epoch(tl, stage)
        print(f"{tag} epoch {ep}: {' '.join(f'{v:.9g}' for v in tup)}", flush=True)


def main():
    mode = sys.argv[1]
    if mode == "poison":
        import contextlib
        import io
        for st in (2, 4):
            for bs in (1, 2):
                for p in (False, True):
                    with contextlib.redirect_stdout(io.StringIO()) as buf:
                        run(bs, f"s{st} bs{bs} {'poison' if p else 'plain'}", poison=p, stage=st,
                            epochs=2)
                    print("\n".join(l for l in buf.getvalue().splitlines() if l.startswith("s")),
                          flush=True)
    elif mode == "single":
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()) as buf:
            run(1, "single")
        print("\n".join(l for l in buf.getvalue().splitlines() if l.startswith("single")))
    elif mode == "rank":
        import torch.distributed as dist
        import torch
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
        run(2, f"rank{os.environ['RANK']}")
        dist.barrier()
        dist.destroy_process_group()
    else:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2",
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs = [subprocess.Popen([sys.executable, "-u", __file__, "rank"],
                                  env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), cwd=str(ROOT),
                                  stdout=subprocess.PIPE, text=True)
                 for r in range(2)]
        outs = [p.communicate(timeout=400)[0] for p in procs]
        for o in outs:
            print("\n".join(l for l in o.splitlines() if l.startswith("rank")))
        sys.exit(max(p.returncode for p in procs))


if __name__ == "__main__":
    main()
