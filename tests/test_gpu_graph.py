"""A whole training step captured as a HIP graph (ctn_graph.StepGraph) against the same
steps run eagerly: after warmup + replays the parameters, Adam moments and loss equal the
eager run's bit for bit (the same kernels on the same values; Adam(capturable=True) reads
its step count and bias corrections from device memory, ctn_adam_step_dev).  Also:
capturable Adam alone against the eager Adam over several steps, and its state_dict step
counts.  GPU only.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(seed, capturable):
    import conv_tasnet as ct
    import ctn_optim
    import synthetic
    torch.manual_seed(seed)
    model = ct.ConvTasNet(N=64, L=20, B=64, H=128, P=3, X=2, R=2, C=2, norm_type="gLN").cuda()
    model.act_dtype = torch.bfloat16
    opt = ctn_optim.Adam(model.parameters(), lr=1e-3, capturable=capturable)
    mix, src = synthetic.speech_like(4, 2, 4000, 11)
    return model, opt, mix.cuda(), src.cuda(), torch.full((4,), 4000, dtype=torch.int64, device="cuda")


def _step_fn(model, opt, mix, src, lens):
    import ctn_optim
    import pit_criterion as pc

    def step():
        est = model(mix)
        loss = pc.cal_loss(src, est, lens)[0]
        opt.zero_grad(set_to_none=True)
        loss.backward()
        ctn_optim.clip_grad_norm_(model.parameters(), 5.0)
        opt.step()
        return loss
    return step


@pytest.mark.timeout(300)
def test_graph_replay_equals_eager_steps():
    import ctn_graph
    eager = _setup(3, capturable=False)
    graph = _setup(3, capturable=True)
    for a, b in zip(eager[0].parameters(), graph[0].parameters()):
        assert torch.equal(a, b)
    f_e = _step_fn(*eager)
    losses_e = [f_e().detach().clone() for _ in range(5)]
    g = ctn_graph.StepGraph(_step_fn(*graph), warmup=2)     # 2 eager steps, then capture
    losses_g = [g.replay().detach().clone() for _ in range(3)]
    torch.cuda.synchronize()
    assert torch.equal(torch.stack(losses_e[2:]), torch.stack(losses_g))
    for (n, a), b in zip(eager[0].named_parameters(), graph[0].parameters()):
        assert torch.equal(a, b), n
    sd_e, sd_g = eager[1].state_dict(), graph[1].state_dict()
    for k in sd_e["state"]:
        assert float(sd_e["state"][k]["step"]) == float(sd_g["state"][k]["step"]) == 5.0
        assert torch.equal(sd_e["state"][k]["exp_avg"], sd_g["state"][k]["exp_avg"])
        assert torch.equal(sd_e["state"][k]["exp_avg_sq"], sd_g["state"][k]["exp_avg_sq"])


def test_capturable_adam_matches_eager_adam():
    import ctn_optim
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s, device="cuda")) for s in [(512, 256), (7,), (1,), (100003,)]]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    oa = ctn_optim.Adam(ps, lr=2e-3, weight_decay=1e-4, capturable=True)
    ob = ctn_optim.Adam(qs, lr=2e-3, weight_decay=1e-4)
    for step in range(6):
        for a, b in zip(ps, qs):
            g = torch.randn_like(a)
            a.grad, b.grad = g.clone(), g.clone()
        oa.step()
        ob.step()
        for a, b in zip(ps, qs):
            assert torch.equal(a, b), step
    assert [float(s["step"]) for s in oa.state_dict()["state"].values()] == [6.0] * 4
    # a resumed capturable optimizer continues the count
    oc = ctn_optim.Adam([torch.nn.Parameter(p.detach().clone()) for p in ps], lr=2e-3, weight_decay=1e-4,
                        capturable=True)
    oc.load_state_dict(copy.deepcopy(oa.state_dict()))
    assert [float(s["step"]) for s in oc.state_dict()["state"].values()] == [6.0] * 4


def test_capturable_adam_no_step_limit_and_lr_changes():
    """the capturable Adam reads no table — past the old 2^20-step table it still
    updates, bit for bit as the eager Adam at the same step count — and an lr change
    between steps reaches its device lr (both paths compute the bias corrections with the
    same device code, ctn_optim.hip adam_bias)."""
    import ctn_optim
    torch.manual_seed(1)
    ps = [torch.nn.Parameter(torch.randn(s, device="cuda")) for s in [(300, 7), (5,)]]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    oa = ctn_optim.Adam(ps, lr=1e-3, capturable=True)
    ob = ctn_optim.Adam(qs, lr=1e-3)
    for a, b in zip(ps, qs):
        a.grad = torch.ones_like(a)
        b.grad = torch.ones_like(b)
    oa.step()
    ob.step()
    big = (1 << 21) + 3
    for o in (oa, ob):
        sd = copy.deepcopy(o.state_dict())
        for st in sd["state"].values():
            st["step"] = torch.tensor(float(big))
        o.load_state_dict(sd)
    for step in range(4):
        if step == 2:
            for o in (oa, ob):
                o.param_groups[0]["lr"] = 3e-4
        before = [a.detach().clone() for a in ps]
        for a, b in zip(ps, qs):
            g = torch.randn_like(a)
            a.grad, b.grad = g.clone(), g.clone()
        oa.step()
        ob.step()
        for a, b, a0 in zip(ps, qs, before):
            assert torch.equal(a, b), step
            assert not torch.equal(a, a0), step          # the update happened
    assert [float(s["step"]) for s in oa.state_dict()["state"].values()] == [float(big + 4)] * 2
    assert float(oa.lr_tensor(0)) == pytest.approx(3e-4)
