"""apex.RNN — experimental stacked / bidirectional RNNs with fused HIP cells (R-23..R-27)."""
from .models import GRU, LSTM, ReLU, Tanh, mLSTM, mLSTMRNNCell
from .RNNBackend import RNNCell, bidirectionalRNN, stackedRNN

__all__ = ["LSTM", "GRU", "ReLU", "Tanh", "mLSTM", "mLSTMRNNCell", "RNNCell", "stackedRNN",
           "bidirectionalRNN"]
