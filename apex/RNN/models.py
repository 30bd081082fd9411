"""apex.RNN model factories (R-26): LSTM, GRU, ReLU, Tanh, mLSTM.

Reference signature (apex/RNN/models.py:19-52):
``X(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0,
bidirectional=False, output_size=None)``.
"""
from __future__ import annotations

import torch.nn as nn

from .cells import GRUCell, LSTMCell, RNNReLUCell, RNNTanhCell, mLSTMCell
from .RNNBackend import RNNCell, bidirectionalRNN, stackedRNN


def toRNNBackend(inputRNN, num_layers, bidirectional=False, dropout=0):
    if bidirectional:
        return bidirectionalRNN(inputRNN, num_layers, dropout=dropout)
    return stackedRNN(inputRNN, num_layers, dropout=dropout)


def LSTM(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0,
         bidirectional=False, output_size=None):
    cell = RNNCell(4, input_size, hidden_size, LSTMCell, 2, bias, output_size)
    return toRNNBackend(cell, num_layers, bidirectional, dropout=dropout)


def GRU(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0,
        bidirectional=False, output_size=None):
    cell = RNNCell(3, input_size, hidden_size, GRUCell, 1, bias, output_size)
    return toRNNBackend(cell, num_layers, bidirectional, dropout=dropout)


def ReLU(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0,
         bidirectional=False, output_size=None):
    cell = RNNCell(1, input_size, hidden_size, RNNReLUCell, 1, bias, output_size)
    return toRNNBackend(cell, num_layers, bidirectional, dropout=dropout)


def Tanh(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0,
         bidirectional=False, output_size=None):
    cell = RNNCell(1, input_size, hidden_size, RNNTanhCell, 1, bias, output_size)
    return toRNNBackend(cell, num_layers, bidirectional, dropout=dropout)


class mLSTMRNNCell(RNNCell):
    """Multiplicative-LSTM cell (reference apex/RNN/cells.py:12-53)."""

    def __init__(self, input_size, hidden_size, bias=False, output_size=None):
        super().__init__(4, input_size, hidden_size, mLSTMCell, n_hidden_states=2, bias=bias,
                         output_size=output_size)
        self.w_mih = nn.Parameter(self.w_ih.new_empty(self.output_size, self.input_size))
        self.w_mhh = nn.Parameter(self.w_ih.new_empty(self.output_size, self.output_size))
        self.reset_parameters()

    def _run_cell(self, input, hidden_state):
        return self.cell(input, hidden_state, self.w_ih, self.w_hh, self.w_mih, self.w_mhh,
                         b_ih=self.b_ih, b_hh=self.b_hh)

    def new_like(self, new_input_size=None):
        if new_input_size is None:
            new_input_size = self.input_size
        return type(self)(new_input_size, self.hidden_size, self.bias, self.output_size)


def mLSTM(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0,
          bidirectional=False, output_size=None):
    cell = mLSTMRNNCell(input_size, hidden_size, bias=bias, output_size=output_size)
    return toRNNBackend(cell, num_layers, bidirectional, dropout=dropout)
