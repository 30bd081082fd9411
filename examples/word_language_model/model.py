"""RNN language model: embedding -> LSTM/GRU/RNN -> (tied) decoder.

``backend="torch"`` runs the recurrent stack through torch.nn (MIOpen RNN kernels on MI355X);
``backend="apex"`` builds it from apex.RNN, whose LSTM/GRU cells use the fused HIP pointwise
kernels (K-06). Under amp O1 the torch path is cast by the RNN compat shim (R-07)."""
from __future__ import annotations

import torch
import torch.nn as nn

import apex.RNN as arnn


class RNNModel(nn.Module):
    def __init__(self, rnn_type, ntoken, ninp, nhid, nlayers, dropout=0.5, tie_weights=False, backend="torch"):
        super().__init__()
        self.drop = nn.Dropout(dropout)
        self.encoder = nn.Embedding(ntoken, ninp)
        self.backend = backend
        if backend == "apex":
            factory = {"LSTM": arnn.LSTM, "GRU": arnn.GRU, "RNN_TANH": arnn.Tanh, "RNN_RELU": arnn.ReLU}[rnn_type]
            self.rnn = factory(ninp, nhid, nlayers, dropout=dropout)
        elif rnn_type in ("LSTM", "GRU"):
            self.rnn = getattr(nn, rnn_type)(ninp, nhid, nlayers, dropout=dropout)
        else:
            nl = {"RNN_TANH": "tanh", "RNN_RELU": "relu"}[rnn_type]
            self.rnn = nn.RNN(ninp, nhid, nlayers, nonlinearity=nl, dropout=dropout)
        self.decoder = nn.Linear(nhid, ntoken)
        if tie_weights:
            if nhid != ninp:
                raise ValueError("When using the tied flag, nhid must be equal to emsize")
            self.decoder.weight = self.encoder.weight
        r = 0.1
        nn.init.uniform_(self.encoder.weight, -r, r)
        nn.init.zeros_(self.decoder.bias)
        if not tie_weights:
            nn.init.uniform_(self.decoder.weight, -r, r)
        self.rnn_type, self.nhid, self.nlayers = rnn_type, nhid, nlayers

    def forward(self, input, hidden):
        emb = self.drop(self.encoder(input))
        if self.backend == "apex":  # state lives in the apex cells (detach_hidden between batches)
            output, _ = self.rnn(emb)
        else:
            output, hidden = self.rnn(emb, hidden)
        output = self.drop(output)
        return self.decoder(output), hidden

    def init_hidden(self, bsz):
        w = next(self.parameters())
        z = lambda: w.new_zeros(self.nlayers, bsz, self.nhid)  # noqa: E731
        if self.backend == "apex":
            self.rnn.reset_hidden(bsz)
            return None
        return (z(), z()) if self.rnn_type == "LSTM" else z()


def repackage_hidden(h, model=None):
    """Detach hidden state from its history (truncated BPTT)."""
    if h is None:
        if model is not None and model.backend == "apex":
            model.rnn.detach_hidden()
        return None
    if isinstance(h, torch.Tensor):
        return h.detach()
    return type(h)(repackage_hidden(v) for v in h)
