"""CPU: ParamStore flat layout — reverse registration order, 16-B alignment, adjacency groups (wav2vec2 q/k/v,
SwinV2 q_bias | zero gap | v_bias) and SGD runs that never cover a gap."""
import torch
import torch.nn as nn

from deepfake_amd.params import ParamStore


class _Attn(nn.Module):
    def __init__(self, C):
        super().__init__()
        self.k_proj, self.v_proj, self.q_proj = nn.Linear(C, C), nn.Linear(C, C), nn.Linear(C, C)
        self.q_bias, self.v_bias = nn.Parameter(torch.randn(C)), nn.Parameter(torch.randn(C))
        self.odd = nn.Parameter(torch.randn(5))

    def flat_groups(self):
        q, k, v = self.q_proj, self.k_proj, self.v_proj
        return [[q.weight, k.weight, v.weight], [q.bias, k.bias, v.bias], [self.q_bias, self.q_bias.numel(),
                                                                           self.v_bias]]


def test_groups_adjacent_and_gapped():
    C = 16
    m = nn.Sequential(_Attn(C), _Attn(C))
    ref = {n: p.detach().clone() for n, p in m.named_parameters()}
    st = ParamStore(m, torch.float32)
    for n, p in m.named_parameters():          # values survive the move into the flat buffer
        assert torch.equal(p.detach(), ref[n])
    for i, p in enumerate(st.params):
        assert st.offsets[i] % 8 == 0 or st.offsets[i] == st.offsets[i - 1] + st.params[i - 1].numel()
    a = m[0]
    ws = st.group_span([a.q_proj.weight, a.k_proj.weight, a.v_proj.weight])
    assert ws is not None and ws[1] == 3 * C * C
    W = st.flat[ws[0]:ws[0] + ws[1]].view(3 * C, C)
    assert torch.equal(W, torch.cat((a.q_proj.weight, a.k_proj.weight, a.v_proj.weight)).detach())
    bs = st.group_span([a.q_bias, C, a.v_bias])
    assert bs is not None and bs[1] == 3 * C
    b = st.flat[bs[0]:bs[0] + bs[1]]
    assert torch.equal(b, torch.cat((a.q_bias, torch.zeros(C), a.v_bias)).detach())
    # a span in the wrong order is not a group
    assert st.group_span([a.k_proj.weight, a.q_proj.weight, a.v_proj.weight]) is None
    # SGD runs cover every parameter and never the gap
    st.touched = [True] * len(st.params)
    runs = st.touched_runs()
    gap = set(range(bs[0] + C, bs[0] + 2 * C))
    covered = set()
    for s, e, _ in runs:
        covered |= set(range(s, e))
    assert not (covered & gap)
    for i, p in enumerate(st.params):
        assert set(range(st.offsets[i], st.offsets[i] + p.numel())) <= covered
    # gradients are views of the flat gradient buffer
    assert a.q_bias.grad.data_ptr() == st.grad[bs[0]:].data_ptr()
