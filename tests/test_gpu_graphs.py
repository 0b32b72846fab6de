"""The opt-in hipGraph mode of the trainer step (ugpg.graphs, trainer.enable_graphs): a
replayed step computes exactly what the eager step computes from the same state, over
several steps with changing data, across a hyperparameter change and a change of the
frozen previous stage (both capture again), with eager steps in between (bench.py's
sampled roofline steps), under both arithmetics."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(dev, res):
    import ugpg
    torch.manual_seed(1234)
    tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device=dev, uncertainty_alpha=1.0)
    tr.stage_configs[3]["resolution"], tr.stage_configs[4]["resolution"] = res // 2, res
    tr.current_stage, tr.current_model = 4, tr.models[4]
    tr.setup_optimizer(4)
    tr.current_model.train()
    tr.models[3].eval()
    return tr


def _state(tr):
    m = tr.current_model
    out = [t.detach().clone() for t in m.state_dict().values()]
    for p in m.parameters():
        st = tr.optimizer.state[p]
        out += [st["square_avg"].clone(), st["step"].clone(), p.grad.clone()]
    return out


def _equal(a, b):
    sa, sb = _state(a), _state(b)
    assert len(sa) == len(sb)
    for i, (u, v) in enumerate(zip(sa, sb)):
        assert torch.equal(u, v), f"state tensor {i} differs"


@pytest.mark.parametrize("math", ["x6", "bf16"])
def test_graphed_train_step_equals_eager(dev, math):
    from ugpg import ops
    old = ops.conv_math()
    ops.set_conv_math(math)
    try:
        res, B = 64, 2
        A, G = _make(dev, res), _make(dev, res)
        G.enable_graphs()
        gen = torch.Generator().manual_seed(7)
        batches = [(torch.randn(B, 3, res, res, generator=gen).to(dev),
                    (torch.rand(B, 1, res, res, generator=gen) < 0.5).float().to(dev))
                   for _ in range(10)]

        def step(k):
            x, t = batches[k]
            ma, mg = A.train_step(x, t, 4).tolist(), G.train_step(x, t, 4).tolist()
            assert ma == mg, (k, ma, mg)

        step(0)  # eager (the key's first step)
        assert G.last_step_graph is None
        step(1)  # captures and replays
        graph = G.last_step_graph
        step(2)  # replays
        assert graph is not None and G.last_step_graph is graph and graph.replays == 2
        _equal(A, G)
        # an eager step in between (what bench.py's timed roofline steps do)
        ops.TIMER = ops.KernelTimer()
        try:
            step(3)
        finally:
            ops.TIMER = None
        assert graph.replays == 2
        step(4)
        assert graph.replays == 3
        _equal(A, G)
        # a hyperparameter change: eager once, then a new capture
        for tr in (A, G):
            for grp in tr.optimizer.param_groups:
                grp["lr"] = 3e-4
        step(5)
        assert G.last_step_graph is None
        step(6)
        assert G.last_step_graph is not None and G.last_step_graph is not graph
        # so does a change of the frozen previous stage (it produces the uncertainty map)
        with torch.no_grad():
            for tr in (A, G):
                next(tr.models[3].parameters()).mul_(0.5)
        graph = G.last_step_graph
        step(7)
        assert G.last_step_graph is None
        step(8)
        assert G.last_step_graph is not None and G.last_step_graph is not graph
        assert len(G._graphs) == G.GRAPH_SLOTS
        step(9)
        _equal(A, G)
        # an epoch's last, shorter batch: its own capture beside the full batches' one
        full = G.last_step_graph
        for k in range(3):
            x, t = batches[k]
            ma, mg = A.train_step(x[:1], t[:1], 4).tolist(), G.train_step(x[:1], t[:1], 4).tolist()
            assert ma == mg, ("short batch", k, ma, mg)
        assert G.last_step_graph is not None and G.last_step_graph is not full
        step(0)
        assert G.last_step_graph is full
        _equal(A, G)
    finally:
        ops.TIMER = None
        ops.set_conv_math(old)
