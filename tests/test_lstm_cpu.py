"""GkLSTM (ops/lstm.py) on the CPU: the same recurrence as nn.LSTM (fp32
fallback of the fused cell), forward and every gradient, and the PTB model
stepping through the compressed optimizer."""
import torch

from gaussiank_sgd_amd.ops.lstm import GkLSTM


def test_gklstm_matches_nn_lstm():
    torch.manual_seed(0)
    T, B, I, H, L = 5, 3, 6, 8, 2
    ref = torch.nn.LSTM(I, H, num_layers=L)
    m = GkLSTM(I, H, num_layers=L)
    assert list(m.state_dict()) == list(ref.state_dict())
    m.load_state_dict(ref.state_dict())
    x = torch.randn(T, B, I, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    h0 = (torch.randn(L, B, H, requires_grad=True), torch.randn(L, B, H, requires_grad=True))
    h0r = tuple(t.detach().clone().requires_grad_(True) for t in h0)
    y, (hn, cn) = m(x, h0)
    yr, (hnr, cnr) = ref(x2, h0r)
    assert torch.allclose(y, yr, atol=1e-5) and torch.allclose(hn, hnr, atol=1e-5) and torch.allclose(cn, cnr, atol=1e-5)
    g = torch.randn_like(y)
    ((y * g).sum() + hn.sum() + 2 * cn.sum()).backward()
    ((yr * g).sum() + hnr.sum() + 2 * cnr.sum()).backward()
    assert torch.allclose(x.grad, x2.grad, atol=1e-5)
    assert torch.allclose(h0[0].grad, h0r[0].grad, atol=1e-5) and torch.allclose(h0[1].grad, h0r[1].grad, atol=1e-5)
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-5), n


def test_ptb_lstm_cpu_step():
    from test_linear_cpu import _step
    t = _step("lstm", "ptb", 4)
    assert isinstance(t.net.lstm, GkLSTM)
