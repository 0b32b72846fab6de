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


def test_graphed_step_after_optimizer_state_reload(dev):
    """a captured step writes RMSprop's square_avg through the pointers it
    was captured with.  ``optimizer.load_state_dict`` (resuming from the trainer's own
    checkpoint dict) replaces those tensors: the key (which holds the optimizer and the
    square_avg storages) must not match the old capture, so the next step runs eagerly and
    captures again -- and the state stays equal to the eager trainer's."""
    import copy
    res, B = 64, 2
    A, G = _make(dev, res), _make(dev, res)
    G.enable_graphs()
    gen = torch.Generator().manual_seed(11)
    batches = [(torch.randn(B, 3, res, res, generator=gen).to(dev),
                (torch.rand(B, 1, res, res, generator=gen) < 0.5).float().to(dev))
               for _ in range(7)]

    def step(k):
        x, t = batches[k]
        ma, mg = A.train_step(x, t, 4).tolist(), G.train_step(x, t, 4).tolist()
        assert ma == mg, (k, ma, mg)

    for k in range(3):
        step(k)
    old = G.last_step_graph
    assert old is not None and old.replays == 2
    for tr in (A, G):  # a resume: the saved optimizer state, loaded back (new tensors)
        tr.optimizer.load_state_dict(copy.deepcopy(tr.optimizer.state_dict()))
    step(3)
    assert G.last_step_graph is None  # the old capture is not replayed
    step(4)
    step(5)
    assert G.last_step_graph is not None and G.last_step_graph is not old
    _equal(A, G)
    # a new optimizer for the same stage (setup_optimizer) drops every capture
    for tr in (A, G):
        tr.setup_optimizer(4)
    assert len(G._graphs) == 0 and G.last_step_graph is None
    step(6)
    _equal(A, G)


def test_graphed_progressive_epochs_equal_eager(dev, tmp_path):
    """the real epoch loop under UGPG_GRAPHS -- train_progressive over two
    stages (transfer_weights + setup_optimizer between them), each epoch's training steps
    replayed, eval-mode validation passes between epochs (eager, no_grad), the stage-end
    BatchNorm buffers -- gives the eager run's weights, BatchNorm buffers and history."""
    import ugpg
    from torch.utils.data import DataLoader, TensorDataset
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(8, 3, 64, 64, generator=gen)
    t = (torch.rand(8, 1, 64, 64, generator=gen) < 0.3).float()
    runs = []
    for graphs in (False, True):
        torch.manual_seed(99)
        tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device=dev, uncertainty_alpha=1.0)
        for s in tr.stage_configs:
            tr.stage_configs[s]["epochs_per_stage"] = 2
        tr.enable_graphs(graphs)
        loader = DataLoader(TensorDataset(x, t), batch_size=2, shuffle=False)
        tr.train_progressive(loader, loader, max_stages=2, save_dir=str(tmp_path / f"g{int(graphs)}"))
        if graphs:
            assert any(g.replays > 0 for g in tr._graphs.values()), "no step was replayed"
        runs.append(tr)
    e, g = runs
    assert e.history == g.history
    for s in (1, 2):
        for (k, a), (_, b) in zip(e.models[s].state_dict().items(), g.models[s].state_dict().items()):
            assert torch.equal(a, b), (s, k)
