"""apex.RNN backend: RNNCell / stackedRNN / bidirectionalRNN (R-23..R-25).

Same module API as the reference (apex/RNN/RNNBackend.py:25-365): inputs are
[seq, batch, features] (never batch_first), hidden state lives in the cell modules and is
created lazily per batch size. Fixed vs the reference:
``bidirectionalRNN.detach_hidden`` called a nonexistent ``detachHidden``; ``stackedRNN``
built flattened ``[layer, batch, features]`` hiddens and then returned the unflattened
lists — the flattened tensors are returned here.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def is_iterable(maybe_iterable):
    return isinstance(maybe_iterable, (list, tuple))


def flatten_list(tens_list):
    """list of [bsz, feat] tensors -> Tensor[len, bsz, feat]."""
    if not is_iterable(tens_list):
        return tens_list
    return torch.stack(list(tens_list), 0)


class bidirectionalRNN(nn.Module):
    def __init__(self, inputRNN, num_layers=1, dropout=0):
        super().__init__()
        self.dropout = dropout
        self.fwd = stackedRNN(inputRNN, num_layers=num_layers, dropout=dropout)
        self.bckwrd = stackedRNN(inputRNN.new_like(), num_layers=num_layers, dropout=dropout)
        self.rnns = nn.ModuleList([self.fwd, self.bckwrd])

    def forward(self, input, collect_hidden=False):
        fwd_out, fwd_hiddens = self.fwd(input, collect_hidden=collect_hidden)
        bck_out, bck_hiddens = self.bckwrd(input, reverse=True, collect_hidden=collect_hidden)
        output = torch.cat([fwd_out, bck_out], -1)
        if collect_hidden:
            hiddens = tuple([torch.cat([a, b], -1) for a, b in zip(fh, bh)]
                            for fh, bh in zip(fwd_hiddens, bck_hiddens))
        else:
            hiddens = tuple(torch.cat([a, b], -1) for a, b in zip(fwd_hiddens, bck_hiddens))
        return output, hiddens

    def reset_parameters(self):
        for rnn in self.rnns:
            rnn.reset_parameters()

    def init_hidden(self, bsz):
        for rnn in self.rnns:
            rnn.init_hidden(bsz)

    def detach_hidden(self):
        for rnn in self.rnns:
            rnn.detach_hidden()

    def reset_hidden(self, bsz):
        for rnn in self.rnns:
            rnn.reset_hidden(bsz)

    def init_inference(self, bsz):
        for rnn in self.rnns:
            rnn.init_inference(bsz)


class stackedRNN(nn.Module):
    """Stack of cells run step by step (the reference's Python time loop).

    ``forward(input[seq, bsz, feat])`` -> (output[seq, bsz, out], hiddens) where hiddens is
    a list over hidden-state kinds of Tensor[layer, bsz, feat] (or, with
    ``collect_hidden``, a list over kinds of per-step Tensor[layer, bsz, feat]).
    """

    def __init__(self, inputRNN, num_layers=1, dropout=0):
        super().__init__()
        self.dropout = dropout
        if isinstance(inputRNN, RNNCell):
            self.rnns = [inputRNN]
            for _ in range(num_layers - 1):
                self.rnns.append(inputRNN.new_like(inputRNN.output_size))
        elif isinstance(inputRNN, list):
            assert len(inputRNN) == num_layers, "RNN list length must be equal to num_layers"
            self.rnns = inputRNN
        else:
            raise RuntimeError("stackedRNN expects an RNNCell or a list of layers")
        self.nLayers = len(self.rnns)
        self.rnns = nn.ModuleList(self.rnns)

    def forward(self, input, collect_hidden=False, reverse=False):
        seq_len = input.size(0)
        steps = reversed(range(seq_len)) if reverse else range(seq_len)
        per_layer = [[] for _ in range(self.nLayers)]
        outputs = []
        for t in steps:
            prev = input[t]
            for layer in range(self.nLayers):
                outs = self.rnns[layer](prev)
                if collect_hidden or t == (0 if reverse else seq_len - 1):
                    per_layer[layer].append(outs)
                prev = outs[0]
                if self.dropout and self.training and layer < self.nLayers - 1:
                    prev = F.dropout(prev, self.dropout, True)
            outputs.append(prev)
        if reverse:
            outputs = list(reversed(outputs))
        output = flatten_list(outputs)
        n_hid = self.rnns[0].n_hidden_states
        steps_kept = len(per_layer[0])
        hiddens = []
        for i in range(n_hid):
            per_step = [flatten_list([per_layer[k][j][i] for k in range(self.nLayers)])
                        for j in range(steps_kept)]
            if reverse:
                per_step = list(reversed(per_step))
            hiddens.append(per_step if collect_hidden else per_step[0])
        return output, hiddens

    def reset_parameters(self):
        for rnn in self.rnns:
            rnn.reset_parameters()

    def init_hidden(self, bsz):
        for rnn in self.rnns:
            rnn.init_hidden(bsz)

    def detach_hidden(self):
        for rnn in self.rnns:
            rnn.detach_hidden()

    def reset_hidden(self, bsz):
        for rnn in self.rnns:
            rnn.reset_hidden(bsz)

    def init_inference(self, bsz):
        for rnn in self.rnns:
            rnn.init_inference(bsz)


class RNNCell(nn.Module):
    """Generic gated cell (``gate_multiplier`` = 4 for LSTM, 3 for GRU, 1 for Elman).

    Parameters ``w_ih [gates*H, in]``, ``w_hh [gates*H, out]``, optional biases and an
    output projection ``w_ho [out, H]`` when ``output_size != hidden_size``.
    """

    def __init__(self, gate_multiplier, input_size, hidden_size, cell, n_hidden_states=2, bias=False,
                 output_size=None):
        super().__init__()
        self.gate_multiplier = gate_multiplier
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.cell = cell
        self.bias = bias
        self.output_size = hidden_size if output_size is None else output_size
        self.gate_size = gate_multiplier * hidden_size
        self.n_hidden_states = n_hidden_states
        self.w_ih = nn.Parameter(torch.empty(self.gate_size, self.input_size))
        self.w_hh = nn.Parameter(torch.empty(self.gate_size, self.output_size))
        if self.output_size != self.hidden_size:
            self.w_ho = nn.Parameter(torch.empty(self.output_size, self.hidden_size))
        self.b_ih = self.b_hh = None
        if self.bias:
            self.b_ih = nn.Parameter(torch.empty(self.gate_size))
            self.b_hh = nn.Parameter(torch.empty(self.gate_size))
        self.hidden = [None for _ in range(self.n_hidden_states)]
        self.reset_parameters()

    def new_like(self, new_input_size=None):
        if new_input_size is None:
            new_input_size = self.input_size
        return type(self)(self.gate_multiplier, new_input_size, self.hidden_size, self.cell,
                          self.n_hidden_states, self.bias, self.output_size)

    def reset_parameters(self, gain=1):
        stdev = 1.0 / math.sqrt(self.hidden_size)
        for p in self.parameters():
            p.data.uniform_(-stdev, stdev)

    def init_hidden(self, bsz):
        ref = next(self.parameters())
        for i in range(len(self.hidden)):
            if self.hidden[i] is None or self.hidden[i].size(0) != bsz:
                size = self.output_size if i == 0 else self.hidden_size
                self.hidden[i] = torch.zeros(bsz, size, dtype=ref.dtype, device=ref.device)

    def reset_hidden(self, bsz):
        self.hidden = [None for _ in self.hidden]
        self.init_hidden(bsz)

    def init_inference(self, bsz):
        self.reset_hidden(bsz)

    def detach_hidden(self):
        if any(h is None for h in self.hidden):
            raise RuntimeError("Must initialize hidden state before you can detach it")
        self.hidden = [h.detach() for h in self.hidden]

    def _run_cell(self, input, hidden_state):
        return self.cell(input, hidden_state, self.w_ih, self.w_hh, b_ih=self.b_ih, b_hh=self.b_hh)

    def forward(self, input):
        self.init_hidden(input.size(0))
        hidden_state = self.hidden[0] if self.n_hidden_states == 1 else tuple(self.hidden)
        out = self._run_cell(input, hidden_state)
        self.hidden = list(out) if self.n_hidden_states > 1 else [out]
        if self.output_size != self.hidden_size:
            self.hidden[0] = F.linear(self.hidden[0], self.w_ho)
        return tuple(self.hidden)
