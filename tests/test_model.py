"""Model / checkpoint-format compatibility with the reference Model."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from pytorch_dppo_amd.models.actor_critic import ActorCritic, pad32


class RefStructuredModel(nn.Module):
    """Same module/parameter structure as the reference ``Model`` (model.py:8-45), written
    independently for the test: layers built in the same order, biases zeroed, log_std zero."""

    def __init__(self, O, A, h=100):
        super().__init__()
        self.p_fc1 = nn.Linear(O, h)
        self.p_fc2 = nn.Linear(h, h)
        self.v_fc1 = nn.Linear(O, h * 5)
        self.v_fc2 = nn.Linear(h * 5, h)
        self.mu = nn.Linear(h, A)
        self.log_std = nn.Parameter(torch.zeros(1, A))
        self.v = nn.Linear(h, 1)
        for name, prm in self.named_parameters():
            if "bias" in name:
                prm.data.fill_(0)

    def forward(self, x):
        h = torch.tanh(self.p_fc2(torch.tanh(self.p_fc1(x))))
        g = torch.tanh(self.v_fc2(torch.tanh(self.v_fc1(x))))
        return self.mu(h), torch.exp(self.log_std), self.v(g)


def test_state_dict_keys_shapes_order_match_reference():
    ref = RefStructuredModel(376, 17)
    ours = ActorCritic(376, 17)
    rk = [(k, tuple(v.shape)) for k, v in ref.state_dict().items()]
    ok = [(k, tuple(v.shape)) for k, v in ours.state_dict().items()]
    assert rk == ok
    assert ok[0][0] == "log_std"
    assert ours.num_params == 288235  # SURVEY §2.6 Humanoid


def test_same_seed_same_init_and_forward_as_reference():
    torch.manual_seed(1)
    ref = RefStructuredModel(17, 6)
    torch.manual_seed(1)
    ours = ActorCritic(17, 6)
    for (k1, v1), (k2, v2) in zip(ref.state_dict().items(), ours.state_dict().items()):
        assert k1 == k2 and torch.equal(v1, v2), k1
    x = torch.randn(9, 17)
    mu_r, s_r, v_r = ref(x)
    mu, s, v = ours.reference_forward(x)
    assert torch.allclose(mu, mu_r) and torch.allclose(s, s_r) and torch.allclose(v, v_r)


def test_model_pt_round_trip_strict_into_reference(tmp_path):
    ours = ActorCritic(11, 3)
    with torch.no_grad():
        ours.flat.normal_()
    torch.save(ours.state_dict(), tmp_path / "model.pt")
    sd = torch.load(tmp_path / "model.pt", weights_only=True)
    ref = RefStructuredModel(11, 3)
    ref.load_state_dict(sd, strict=True)
    back = ActorCritic(11, 3)
    back.load_state_dict(ref.state_dict(), strict=True)
    assert torch.equal(back.flat, ours.flat)


def test_grads_flow_into_flat_buffer_contiguously():
    m = ActorCritic(4, 2, hidden=(8, 8))
    mu, ls, v = m(torch.randn(5, 4))
    (mu.sum() + v.sum() + ls.sum()).backward()
    assert m.flat.grad is not None and m.flat.grad.shape == m.flat.shape
    assert torch.all(m.view("log_std", m.flat.grad) == 1.0)   # log_std [1,A] summed once
    assert torch.all(m.view("v.bias", m.flat.grad) == 5.0)     # 5 rows


def test_packed_layout_padded_math_equals_unpadded():
    """The kernels' padded GEMM (bias folded in column K, constant-1 input column) must
    reproduce the unpadded forward exactly — checked here with torch matmuls on the images."""
    torch.manual_seed(0)
    m = ActorCritic(17, 6, hidden=(100, 100))
    L = m.packed_layout()
    img = L.pack(m.flat.data)
    x = torch.randn(7, 17)

    def run(head):
        h = x
        for ls in head:
            Wp = L.image_w(img, ls.name)
            if ls.name not in L.NO_WT:     # (no dgrad into the observations: no transposed image)
                Wpt = L.image_wt(img, ls.name)
                assert torch.equal(Wpt, Wp.t())
            xa = torch.zeros(h.shape[0], ls.d_in)
            xa[:, :ls.fan_in] = h
            xa[:, ls.fan_in] = 1.0
            out = xa @ Wp.t()
            assert torch.all(out[:, ls.fan_out:] == 0)
            h = out[:, :ls.fan_out]
            if ls.act == "tanh":
                h = torch.tanh(h)
        return h

    mu_ref, _, v_ref = m(x)
    assert torch.allclose(run(m.policy_layers), mu_ref, atol=1e-6)
    assert torch.allclose(run(m.value_layers), v_ref, atol=1e-6)
    assert all(ls.d_in % 32 == 0 and ls.d_in > ls.fan_in for ls in L.layers)
    assert pad32(377) == 384


def test_fragment_major_index_is_a_bijection_with_contiguous_fragments():
    from pytorch_dppo_amd.models.actor_critic import fm_index
    rows, cols = 48, 96
    r = torch.arange(rows).repeat_interleave(cols)
    c = torch.arange(cols).repeat(rows)
    idx = fm_index(r, c, cols)
    assert torch.equal(torch.sort(idx).values, torch.arange(rows * cols))
    # lane l of block (rt=1, ks=2) owns row 16 + l%16, cols 64 + 8*(l//16) .. +7 -> offsets base + 8l .. 8l+7
    base = (1 * (cols // 32) + 2) * 512
    for lane in (0, 5, 17, 63):
        rr = torch.full((8,), 16 + lane % 16)
        cc = 64 + 8 * (lane // 16) + torch.arange(8)
        assert torch.equal(fm_index(rr, cc, cols), base + 8 * lane + torch.arange(8))
