"""torch-version helpers (R-10). torch >= 2 only: tensors and Variables are one type."""
import torch


def variable_is_tensor():
    return True


def tensor_is_variable():
    return False


def tensor_is_float_tensor():
    return False


def is_tensor_like(x):
    return torch.is_tensor(x)


def is_floating_point(x):
    return torch.is_tensor(x) and x.is_floating_point()


def scalar_python_val(x):
    return x.item() if hasattr(x, "item") else x[0]
