"""Model zoo for the BASELINE.json configurations (random init, synthetic data):
BERT-Large pretraining (headline), GPT-2 1.5B, Megatron TP/PP GPT, ResNet-50, 2-layer MLP."""
from .bert import BertConfig, BertForPreTraining, BertModel
from .gpt import GPTConfig, GPTModel
from .mlp import MLP
from .resnet import resnet18, resnet34, resnet50, resnet101, resnet152

__all__ = ["BertConfig", "BertForPreTraining", "BertModel", "GPTConfig", "GPTModel", "MLP",
           "resnet18", "resnet34", "resnet50", "resnet101", "resnet152"]
