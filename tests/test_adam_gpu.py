"""Fused Adam kernels against torch.optim.Adam (BS/trainers/base.py:225-228 builds torch.optim.Adam; the
fused step replaces it): rs_adam_prepare_step (one launch) == rs_adam_prepare + rs_adam_step bit for bit,
both within fp32 rounding of torch's update, step count / dropout seed / arrival counter bookkeeping."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _state():
    return torch.zeros(144, dtype=torch.float64, device="cuda")


@pytest.mark.parametrize("n", [1, 7, 4096 + 3, 662_019])
@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_fused_prepare_step_matches_two_launches_and_torch(n, wd):
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    g0 = torch.Generator().manual_seed(n)
    p0 = torch.randn(n, generator=g0)
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, wd], dtype=torch.float64, device="cuda")
    div = torch.tensor([3.0], device="cuda")
    runs = []
    for fused in (False, True):
        p, m, v = p0.cuda().clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
        pb = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        st, seed = _state(), torch.zeros(1, dtype=torch.int64, device="cuda")
        gg = torch.Generator().manual_seed(1)
        for _ in range(5):
            g = torch.randn(n, generator=gg).cuda() * 3.0
            if fused:
                ops.adam_prepare_step(p, g, m, v, pb, st, hyper, zero_grad=True, grad_divisor=div, seed_base=seed)
            else:
                ops.adam_prepare(st, hyper, div, seed)
                ops.adam_step(p, g, m, v, pb, st, hyper, zero_grad=True)
            assert int(torch.count_nonzero(g)) == 0
        torch.cuda.synchronize()
        runs.append((p.clone(), pb.clone(), st.cpu(), int(seed.item())))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])
    assert runs[1][2][0].item() == 5.0 and runs[1][2][7].item() == 0.0 and not runs[1][2][16:].any() and runs[1][3] == 5
    assert torch.equal(runs[0][2][:4], runs[1][2][:4])
    # torch.optim.Adam (L2 weight decay as torch's Adam adds it to the gradient) on the same gradients / 3
    tp = torch.nn.Parameter(p0.clone().double())
    opt = torch.optim.Adam([tp], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd)
    gg = torch.Generator().manual_seed(1)
    for _ in range(5):
        tp.grad = (torch.randn(n, generator=gg) * 3.0 / 3.0).double()
        opt.step()
    err = (runs[1][0].cpu().double() - tp.detach()).abs().max().item()
    assert err < 2e-6, err


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_fused_step_matches_torch_adam_in_float32(wd):
    """The same five steps against torch.optim.Adam on float32 tensors (CPU, the reference's dtype) fed the very
    gradients the kernel uses (g * float(1/divisor)): the moments and the parameters agree to a few float32 ulps.
    The bias corrections and (1 - beta) factors are formed in double and cast to float as torch does with its
    Python-float hyperparameters (fp32 betas put 1 - 0.999f 1.3e-5 relative off torch's float(1 - 0.999): a bias
    in every exp_avg_sq update this bound rejects)."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    n = 100_003
    g0 = torch.Generator().manual_seed(5)
    p0 = torch.randn(n, generator=g0)
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, wd], dtype=torch.float64, device="cuda")
    div = torch.tensor([3.0], device="cuda")
    p, m, v = p0.cuda().clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    st, seed = _state(), torch.zeros(1, dtype=torch.int64, device="cuda")
    tp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([tp], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd, foreach=False)
    gg = torch.Generator().manual_seed(1)
    gs = torch.tensor(1.0, dtype=torch.float32) / torch.tensor(3.0, dtype=torch.float32)
    for _ in range(5):
        g = torch.randn(n, generator=gg) * 3.0
        ops.adam_prepare_step(p, g.cuda(), m, v, None, st, hyper, zero_grad=True, grad_divisor=div, seed_base=seed)
        tp.grad = g * gs
        opt.step()
    torch.cuda.synchronize()
    s = opt.state[tp]

    eps = torch.finfo(torch.float32).eps

    def ulps(a, b):   # elementwise, in float32 ulps of the reference value
        return ((a.double() - b.double()).abs() / eps / b.double().abs().clamp_min(1e-30))

    def ulps_of_max(a, b):   # m and p: signed sums with cancellation -- ulps of the tensor's largest magnitude
        return ((a.double() - b.double()).abs().max() / eps / b.double().abs().max()).item()
    assert ulps(v.cpu(), s["exp_avg_sq"]).max().item() <= 4
    assert ulps_of_max(m.cpu(), s["exp_avg"]) <= 4
    assert ulps_of_max(p.cpu(), tp.detach()) <= 4


@pytest.mark.parametrize("graph", [False, True])
def test_optimizer_written_transposed_weights_match_a_fresh_transpose(graph):
    """SAS fused step: rs_adam_prepare_step writes the backward's transposed bf16 block weights; after
    several steps they equal rs_transpose_bf16 of the current bf16 weights bit for bit."""
    import argparse
    import numpy as np
    import rbm_amd  # noqa: F401
    import rbm_amd.data as synth
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedTrainStep
    torch.manual_seed(0)
    a = argparse.Namespace(model_code="sas", num_items=500, max_len=64, device="cuda", sas_hidden_units=64,
                           sas_num_blocks=2, sas_heads=1, sas_dropout=0.1, l2_emb=0.0, rs_dtype="bf16")
    m = model_factory(a)
    st = FusedTrainStep(m, lr=1e-2)
    rng = np.random.default_rng(0)
    b = [torch.from_numpy(x).cuda() for x in synth.sas_batch(rng, 16, 64, 500)]
    if graph:
        st.capture(*b, warmup=2)
        for _ in range(3):
            st.replay(*b)
    else:
        for _ in range(4):
            st.step(*b)
    torch.cuda.synchronize()
    eng = st.engine
    assert eng.adam_transposes and eng._wT is not None
    got = eng._wT.clone()
    eng.adam_transposes = False
    eng._refresh_transposed()
    torch.cuda.synchronize()
    assert torch.equal(got, eng._wT)


def test_zero_grad_with_untouched_rows():
    """zero_grad stores zeros only where the gradient is not already zero (the untouched rows of a large table keep
    their zeros without a store): with rows of exact zeros (and -0.0) beside non-zero ones, every gradient element
    is zero after the step and the update equals torch.optim.Adam's on the same sparse gradients."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    n, d = 4096 * 64, 64
    gen = torch.Generator().manual_seed(3)
    p0 = torch.randn(n, generator=gen)
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.0], dtype=torch.float64, device="cuda")
    p, m, v = p0.cuda().clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    st, seed = _state(), torch.zeros(1, dtype=torch.int64, device="cuda")
    tp = torch.nn.Parameter(p0.clone().double())
    opt = torch.optim.Adam([tp], lr=1e-3, betas=(0.9, 0.999), eps=1e-8)
    for step in range(3):
        g = torch.randn(n, generator=gen)
        touched = torch.rand(n // d, generator=gen) < 0.2            # 20 % of the rows carry a gradient
        g = (g.view(-1, d) * touched[:, None]).view(-1)
        g[g == 0] = -0.0 if step == 1 else 0.0                       # signed zeros are zeros too
        gd = g.cuda()
        ops.adam_prepare_step(p, gd, m, v, None, st, hyper, zero_grad=True, seed_base=seed)
        torch.cuda.synchronize()
        assert int(torch.count_nonzero(gd)) == 0
        tp.grad = g.double()
        opt.step()
    err = (p.cpu().double() - tp.detach()).abs().max().item()
    assert err < 2e-6, err


def test_step_lr_matches_torch_steplr_and_reaches_captured_graphs():
    """StepLR (BS/trainers/base.py:40, stepped per epoch at :87) through FusedStepLR: (1) the learning rates equal torch's
    StepLR's, and the fused Adam driven by them tracks torch.optim.Adam + StepLR to a few float32 ulps over 4 epochs;
    (2) a FusedTrainStep captured ONCE and replayed across epochs applies each epoch's rate: bit for bit the eager
    steps of a twin trainer under the same schedule, and a zero rate leaves the parameters unchanged."""
    import argparse
    import numpy as np
    import rbm_amd  # noqa: F401
    import rbm_amd.data as synth
    from rbm_amd import ops
    from rbm_amd.models import model_factory
    from rbm_amd.train_step import FusedAdam, FusedStepLR, FusedTrainStep
    n = 50_000
    p0 = torch.randn(n, generator=torch.Generator().manual_seed(2))
    tp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([tp], lr=1e-3, foreach=False)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=2, gamma=0.5)

    class _Flat:
        device = torch.device("cuda")
        numel = n
    fa = FusedAdam(_Flat(), lr=1e-3)
    fs = FusedStepLR(fa, step_size=2, gamma=0.5)
    p, st, seed = p0.cuda().clone(), fa.state, torch.zeros(1, dtype=torch.int64, device="cuda")
    gg = torch.Generator().manual_seed(3)
    for epoch in range(4):
        for _ in range(3):
            g = torch.randn(n, generator=gg)
            ops.adam_prepare_step(p, g.cuda(), fa.m, fa.v, None, st, fa.hyper, zero_grad=True, seed_base=seed)
            tp.grad = g
            opt.step()
        sched.step()
        fs.step()
        assert fs.get_last_lr() == sched.get_last_lr(), (epoch, fs.get_last_lr(), sched.get_last_lr())
        assert float(fa.hyper[0].item()) == sched.get_last_lr()[0]
    torch.cuda.synchronize()
    eps = torch.finfo(torch.float32).eps
    assert ((p.cpu().double() - tp.detach().double()).abs().max() / eps / tp.detach().double().abs().max()) <= 4

    V, T, B = 300, 32, 8
    a = argparse.Namespace(model_code="sas", num_items=V, max_len=T, device="cuda", sas_hidden_units=64,
                           sas_num_blocks=2, sas_heads=1, sas_dropout=0.2, l2_emb=0.0, rs_dtype="bf16")
    rng = np.random.default_rng(4)
    batches = [tuple(torch.from_numpy(x).cuda() for x in synth.sas_batch(rng, B, T, V)) for _ in range(9)]
    runs = []
    for graph in (True, False):
        torch.manual_seed(0)
        m = model_factory(a)
        tr = FusedTrainStep(m, lr=1e-3)
        sch = FusedStepLR(tr, step_size=1, gamma=0.1)
        if graph:
            tr.capture(*batches[0], warmup=1)
        else:
            tr.step(*batches[0])
        snaps = []
        for epoch in range(3):
            for i in range(3):
                b = batches[3 * epoch + i]
                (tr.replay if graph else tr.step)(*b)
            snaps.append(tr.flat.data.clone())
            sch.step()
        sch.optimizer.set_lr(0.0)
        before = tr.flat.data.clone()
        (tr.replay if graph else tr.step)(*batches[0])
        assert torch.equal(tr.flat.data, before), "lr 0 still moved the parameters"
        runs.append(snaps)
    for x, y in zip(*runs):
        assert torch.equal(x, y)


@pytest.mark.parametrize("fused", [False, True])
def test_nontemporal_sweep_matches_the_cached_form(fused):
    """Ranges of >= 64M elements take the nontemporal-hint form of the Adam kernel (misc.hip ADAM_NT_MIN: cfg5's
    out.weight and token-table sweeps); the same elements updated as a shorter range (the cached form) give the same
    bits, zero_grad included, over two steps at a 256-workgroup cap (the early sweeps' grid) and the full grid."""
    import rbm_amd  # noqa: F401
    from rbm_amd import ops
    n, k = (64 << 20) + 4099, 1 << 20
    g0 = torch.Generator(device="cuda").manual_seed(7)
    p = torch.randn(n, generator=g0, device="cuda")
    m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    pb = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.01], dtype=torch.float64, device="cuda")
    div = torch.tensor([2.0], device="cuda")
    # two windows: the head of the range and its ragged tail
    wins = [(0, k), (n - k - 3, n)]
    small = [(p[a:b].clone(), m[a:b].clone(), v[a:b].clone(), torch.empty(b - a, dtype=torch.bfloat16, device="cuda"))
             for a, b in wins]
    st_big, st_small = torch.zeros(144, dtype=torch.float64, device="cuda"), torch.zeros(144, dtype=torch.float64, device="cuda")
    for step in range(2):
        g = torch.randn(n, generator=g0, device="cuda")
        g[: n // 3] = 0.0   # untouched rows keep their zeros without a store
        gs = [g[a:b].clone() for a, b in wins]
        if fused:
            ops.adam_prepare_step(p, g, m, v, pb, st_big, hyper, zero_grad=True, grad_divisor=div)
        else:
            ops.adam_prepare(st_big, hyper, div)
            ops.adam_step(p, g, m, v, pb, st_big, hyper, zero_grad=True, max_wg=256 if step == 0 else None)
        ops.adam_prepare(st_small, hyper, div)
        for (sp, sm, sv, sb), sg in zip(small, gs):
            ops.adam_step(sp, sg, sm, sv, sb, st_small, hyper, zero_grad=True)
        assert int(torch.count_nonzero(g)) == 0
        for (sp, sm, sv, sb), sg in zip(small, gs):
            assert int(torch.count_nonzero(sg)) == 0
    torch.cuda.synchronize()
    for (a, b), (sp, sm, sv, sb) in zip(wins, small):
        assert torch.equal(p[a:b], sp) and torch.equal(m[a:b], sm) and torch.equal(v[a:b], sv)
        assert torch.equal(pb[a:b], sb)
