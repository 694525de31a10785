"""HIP-graph capture of a training step (minips_amd.utils.graph) replays exactly the eager step:
same losses and parameters as the eager model from the same initial state."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_graphed_mlp_matches_eager(dev):
    from minips_amd.data.synthetic import MnistSynth
    from minips_amd.models.mlp import MLP, MLPConfig
    from minips_amd.ps.comm import Comm
    from minips_amd.utils.graph import GraphedStep

    data = MnistSynth(1024, device=dev, seed=4)
    batches = [data.next() for _ in range(10)]
    eager = MLP(MLPConfig(), Comm(device=dev))
    graphed = MLP(MLPConfig(), Comm(device=dev))
    # GraphedStep's 3 warm-up steps are real steps on the example batch (capture runs nothing)
    for _ in range(3):
        eager.train_step(*batches[0])
    step = GraphedStep(lambda x, y: graphed.train_step(x, y)[0], batches[0], tables=[graphed.table])
    le, lg = [], []
    for x, y in batches[1:]:
        le.append(float(eager.train_step(x, y)[0].item()))
        lg.append(float(step(x, y).item()))
    torch.cuda.synchronize()
    assert graphed.table.step == eager.table.step
    assert lg == pytest.approx(le, rel=1e-3, abs=1e-3), (le, lg)
    torch.testing.assert_close(graphed.table.master, eager.table.master, rtol=1e-3, atol=1e-4)


def test_graphed_widedeep_step_matches_eager(dev):
    """The whole one-rank W&D step (data generation + key planning on the planning stream, Get,
    forward/backward with the side stream, Add, Clock) replayed from ONE HIP graph follows the
    eager step: same batches (device-side generator counter), same losses and parameters."""
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.feeder import GraphedFeeder, LookaheadFeeder
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import Comm

    cards = [1000, 50, 20000, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24,
             25, 26]
    runs = {}
    main = torch.cuda.Stream(device=dev)
    main.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(main):
        for mode in ("eager", "graph"):
            model = WideDeep(WideDeepConfig(cards=cards), Comm(device=dev))
            feeder = LookaheadFeeder(model, CriteoSynth(2048, cards=cards, device=dev, seed=3), model.comm, depth=1)
            losses = [float(feeder.step().item()) for _ in range(2)]
            step = GraphedFeeder(feeder, [model.emb, model.dense]).step if mode == "graph" else feeder.step
            for _ in range(6):
                losses.append(float(step().item()))
            torch.cuda.synchronize()
            runs[mode] = (losses, model.dense.master.clone(), model.emb.shard.clone(), model.dense.step)
    (le, de, ee, se), (lg, dg, eg, sg) = runs["eager"], runs["graph"]
    assert se == sg == 8
    assert lg[2] != lg[3]  # replays draw new batches
    assert lg == pytest.approx(le, rel=2e-3, abs=1e-3), (le, lg)
    # float-atomic summation order differs between runs; Adam / row-wise Adagrad normalise the
    # steps, so bound the typical deviation, not the max
    assert float((de - dg).abs().mean()) < 2e-5 and float((ee - eg).abs().mean()) < 1e-4
