"""apex.RNN vs torch.nn RNNs with copied weights (reference tests/RNN/RNN_tests.py, which only
printed differences; here they are asserted). CPU always, GPU (fused HIP cells) with marker."""
import pytest
import torch
from torch import nn

import apex.RNN as RNN

DEVS = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)] if torch.cuda.is_available() else ["cpu"]


def _copy(apex_rnn, torch_rnn, layers, bidir):
    stacks = apex_rnn.rnns if bidir else [apex_rnn]
    for d, stack in enumerate(stacks):
        sfx = "_reverse" if d == 1 else ""
        for k, cell in enumerate(stack.rnns):
            with torch.no_grad():
                cell.w_ih.copy_(getattr(torch_rnn, f"weight_ih_l{k}{sfx}"))
                cell.w_hh.copy_(getattr(torch_rnn, f"weight_hh_l{k}{sfx}"))
                cell.b_ih.copy_(getattr(torch_rnn, f"bias_ih_l{k}{sfx}"))
                cell.b_hh.copy_(getattr(torch_rnn, f"bias_hh_l{k}{sfx}"))


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("kind", ["LSTM", "GRU", "Tanh", "ReLU"])
@pytest.mark.parametrize("layers,bidir", [(1, False), (2, False), (1, True)])  # reference bidir stacks directions independently
def test_rnn_parity(dev, kind, layers, bidir):
    torch.manual_seed(0)
    T, B, I, H = 7, 5, 12, 16
    tmap = {"LSTM": nn.LSTM, "GRU": nn.GRU, "Tanh": lambda *a, **k: nn.RNN(*a, nonlinearity="tanh", **k),
            "ReLU": lambda *a, **k: nn.RNN(*a, nonlinearity="relu", **k)}
    ref = tmap[kind](I, H, num_layers=layers, bidirectional=bidir).to(dev)
    mine = getattr(RNN, kind)(I, H, layers, bidirectional=bidir).to(dev)
    _copy(mine, ref, layers, bidir)
    x = torch.randn(T, B, I, device=dev, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    out, hid = mine(x)
    rout, rhid = ref(x2)
    torch.testing.assert_close(out, rout, rtol=1e-4, atol=1e-5)
    h_ref = rhid[0] if isinstance(rhid, tuple) else rhid
    if bidir:  # torch: [layers*2, B, H] interleaved per direction; ours: [layers, B, 2H]
        h_ref = torch.cat([h_ref[0::2], h_ref[1::2]], -1)
    torch.testing.assert_close(hid[0], h_ref, rtol=1e-4, atol=1e-5)
    (out.sum() + hid[0].sum()).backward()
    (rout.sum() + (rhid[0] if isinstance(rhid, tuple) else rhid).sum()).backward()
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-4, atol=1e-5)
    cell = (mine.rnns[0] if bidir else mine).rnns[0]
    torch.testing.assert_close(cell.w_ih.grad, ref.weight_ih_l0.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(cell.b_hh.grad, ref.bias_hh_l0.grad, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("dev", DEVS)
def test_mlstm_runs_and_matches_manual(dev):
    torch.manual_seed(1)
    m = RNN.mLSTM(6, 8, 1).to(dev)
    x = torch.randn(4, 3, 6, device=dev)
    out, (h, c) = m(x)
    cell = m.rnns[0]
    hx = torch.zeros(3, 8, device=dev)
    cx = torch.zeros(3, 8, device=dev)
    for t in range(4):
        mm = (x[t] @ cell.w_mih.t()) * (hx @ cell.w_mhh.t())
        g = x[t] @ cell.w_ih.t() + cell.b_ih + mm @ cell.w_hh.t() + cell.b_hh
        i, f, gg, o = g.chunk(4, 1)
        cx = torch.sigmoid(f) * cx + torch.sigmoid(i) * torch.tanh(gg)
        hx = torch.sigmoid(o) * torch.tanh(cx)
    torch.testing.assert_close(out[-1], hx, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(c[0], cx, rtol=1e-4, atol=1e-5)


def test_detach_hidden_bidirectional():
    m = RNN.LSTM(4, 4, 1, bidirectional=True)
    m(torch.randn(3, 2, 4))
    m.detach_hidden()  # reference called a nonexistent detachHidden()
