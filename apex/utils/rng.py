"""Seeds for the stateless Philox dropout kernels (attention, bias-dropout-add(-LN)).

The HIP dropout kernels regenerate their masks from a (key, counter-base) pair instead of
storing them. The pair is derived from the device's default torch generator — its seed and
Philox offset — and the offset is advanced by 4 per launch, exactly like a torch dropout op:

* ``torch.manual_seed`` / ``torch.cuda.manual_seed`` make masks reproducible;
* the tensor-parallel RNG tracker (``get_cuda_rng_tracker().fork()``) swaps the device
  generator state, so dropout inside a TP region gets a different key on every TP rank and the
  same key on every DP replica (Megatron semantics; ADVICE r1: the previous CPU-generator draw
  gave every TP rank the same mask);
* ``CheckpointFunction`` restores the device generator state before recomputation, so the
  recomputed forward redraws the same masks.

No device synchronisation: the generator state is host-side.
"""
from __future__ import annotations

import torch

_MASK64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _MASK64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK64
    return z ^ (z >> 31)


def _cuda_seed_offset(idx: int, advance: int):
    gen = torch.cuda.default_generators[idx]
    try:
        seed, off = int(gen.initial_seed()), int(gen.get_offset())
        gen.set_offset(off + advance)
        return seed, off
    except (AttributeError, RuntimeError):
        st = torch.cuda.get_rng_state(idx)  # uint8[16]: seed (u64) then offset (i64)
        seed = int.from_bytes(bytes(st[:8].tolist()), "little")
        off = int.from_bytes(bytes(st[8:16].tolist()), "little")
        new = st.clone()
        new[8:16] = torch.tensor(list((off + advance).to_bytes(8, "little")), dtype=torch.uint8)
        torch.cuda.set_rng_state(new, idx)
        return seed, off


def philox_seed_offset(device=None):
    """(key, counter base) for one dropout launch on ``device``. Two launches never share a
    stream: the key mixes the generator's seed with its (advancing) offset."""
    if device is not None and torch.device(device).type == "cuda":
        dev = torch.device(device)
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        seed, off = _cuda_seed_offset(idx, 4)
        key = _splitmix64(seed ^ _splitmix64(off))
        base = _splitmix64(key ^ 0x5851F42D4C957F2D) & ((1 << 62) - 1)
        return key & ((1 << 62) - 1), base
    s = torch.randint(0, 2 ** 62, (2,), dtype=torch.int64)
    return int(s[0]), int(s[1])
