"""The bandwidth-bound kernels at the benchmark shapes, one op at a time, for rocprofv3 counter
passes (tools/gpu_pmc_bw.sh) and event timing.

    python tools/bw_kernels.py [--ops ln,bdaln,lamb,xent,syncbn,scale] [--iters 5]

Per op prints one JSON line: the kernels it launches, the LOGICAL bytes one call must move
(inputs read once + outputs written once, from the tensor shapes) and the event-timed µs per
call, so the counter totals (FETCH_SIZE / WRITE_SIZE, summarised by tools/pmc_bw_summary.py)
can be set against both.

Shapes: BERT-Large at the headline batch (98304 tokens x 1024 hidden, MLM logits of 768 x 19
masked positions x 30528 vocab, the 336 M-parameter LAMB step with bf16 model copies), ResNet-50's
largest BatchNorm (N 64, C 256, 56 x 56, NCHW bf16).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DEV = "cuda"


def _time(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def op_ln(iters):
    from apex.normalization import FusedLayerNorm

    T, E = 98304, 1024
    ln = FusedLayerNorm(E).to(DEV).bfloat16()
    x = torch.randn(T, E, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn(T, E, device=DEV, dtype=torch.bfloat16)
    y = ln(x)
    fwd = _time(lambda: ln(x), iters)
    bwd = _time(lambda: torch.autograd.grad(y, [x] + list(ln.parameters()), dy, retain_graph=True), iters)
    n = T * E * 2
    return [dict(op="layernorm_fwd", us=fwd, bytes=2 * n + T * 8, kernels="ln_fwd_fast"),
            dict(op="layernorm_bwd", us=bwd, bytes=3 * n + T * 8, kernels="ln_bwd_fast (+ colsum of dgamma/dbeta partials)")]


def op_bdaln(iters):
    import apex._ext as e

    C = e.require()
    T, E = 98304, 1024
    bf = torch.bfloat16
    t = torch.randn(T, E, device=DEV, dtype=bf)
    res = torch.randn(T, E, device=DEV, dtype=bf)
    b = torch.randn(E, device=DEV, dtype=bf)
    g = torch.ones(E, device=DEV, dtype=bf)
    be = torch.zeros(E, device=DEV, dtype=bf)
    y, s, mean, rstd = C.bdaln_fwd(t, b, res, g, be, 1e-12, 0.1, 7, 0)
    dy = torch.randn_like(y)
    fwd = _time(lambda: C.bdaln_fwd(t, b, res, g, be, 1e-12, 0.1, 7, 0), iters)
    bwd = _time(lambda: C.bdaln_bwd(dy, s, g, mean, rstd, 0.1, 7, 0, True), iters)
    n = T * E * 2
    # fwd: read t, res; write y, s (the pre-LN sum kept for backward); bwd: read dy, s; write dres, dt
    return [dict(op="bias_dropout_add_ln_fwd", us=fwd, bytes=4 * n + T * 8, kernels="bdaln_fwd_kernel"),
            dict(op="bias_dropout_add_ln_bwd", us=bwd, bytes=4 * n + T * 8, kernels="bdaln_bwd_kernel")]


def op_lamb(iters):
    from apex import amp
    from apex.amp._amp_state import _amp_state
    from apex.models.bert import BertConfig, BertForPreTraining, param_groups_for_lamb
    from apex.optimizers import FusedLAMB

    _amp_state.optimizers, _amp_state.loss_scalers = [], []
    model = BertForPreTraining(BertConfig.large()).to(DEV)
    opt = FusedLAMB(param_groups_for_lamb(model, 0.01), lr=1e-4, max_grad_norm=1.0)
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
    ps = [p for p in model.parameters()]
    for p in ps:
        p.grad = torch.randn_like(p) * 1e-3
    n = sum(p.numel() for p in ps)
    us = _time(lambda: opt.step(), iters)
    # per parameter: grad-norm pass reads the bf16 grad (2); stage 1 reads g, p, m, v (2 + 12) and
    # writes m, v (8); stage 2 reads p, m, v (12) and writes p (4) + the bf16 model copy (2)
    return [dict(op="fused_lamb_step", us=us, bytes=n * (2 + 14 + 8 + 12 + 6), params=n,
                 kernels="sumsq (grad norm) + lamb_stage1 + lamb_stage2")]


def op_adam(iters):
    """The Megatron GPT (H2560, 32 layers) Adam step: fp32 main_grad, fp32 master, fp32 m / v,
    bf16 model copy — 30 B per parameter, one adam_kernel launch."""
    from apex.multi_tensor_apply import multi_tensor_applier
    from apex.multi_tensor_apply.ops import multi_tensor_adam

    H = 2560
    sizes = ([3 * H * H, 3 * H, H * H, H, 4 * H * H, 4 * H, 4 * H * H, H, H, H, H, H] * 32
             + [50304 * H, 2048 * H, H, H])
    gs = [torch.randn(s, device=DEV) * 1e-3 for s in sizes]
    ps = [torch.randn(s, device=DEV) for s in sizes]
    ms = [torch.zeros(s, device=DEV) for s in sizes]
    vs = [torch.zeros(s, device=DEV) for s in sizes]
    cs = [torch.empty(s, device=DEV, dtype=torch.bfloat16) for s in sizes]
    noop = torch.zeros(1, dtype=torch.int32, device=DEV)
    n = sum(sizes)
    us = _time(lambda: multi_tensor_applier(multi_tensor_adam, noop, [gs, ps, ms, vs, cs], 1e-4, 0.9, 0.999, 1e-8,
                                            1, 1, 1, 0.01), iters)
    return [dict(op="fused_adam_step_megatron", us=us, bytes=n * 30, params=n, kernels="adam_kernel<f32,f32,bf16>")]


def op_xent(iters):
    from apex.contrib.xentropy import softmax_xentropy

    R, V = 768 * 19, 30528
    logits = torch.randn(R, V, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    labels = torch.randint(0, V, (R,), device=DEV)
    loss = softmax_xentropy(logits, labels, 0.0, -100, "mean")
    fwd = _time(lambda: softmax_xentropy(logits, labels, 0.0, -100, "mean"), iters)
    bwd = _time(lambda: torch.autograd.grad(loss, logits, retain_graph=True), iters)
    n = R * V * 2
    return [dict(op="softmax_xentropy_fwd", us=fwd, bytes=n + R * 16, kernels="xent_fwd_kernel"),
            dict(op="softmax_xentropy_bwd", us=bwd, bytes=2 * n + R * 16, kernels="xent_bwd_kernel")]


def op_syncbn(iters, channels_last=False):
    from apex.parallel import SyncBatchNorm

    N, Cc, H, W = 64, 256, 56, 56
    bn = SyncBatchNorm(Cc).to(DEV)
    x = torch.randn(N, Cc, H, W, device=DEV, dtype=torch.bfloat16)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    dy = torch.randn_like(x)
    y = bn(x)
    fwd = _time(lambda: bn(x), iters)
    bwd = _time(lambda: torch.autograd.grad(y, [x] + list(bn.parameters()), dy, retain_graph=True), iters)
    n = x.numel() * 2
    # fwd: stats pass reads x, elementwise pass reads x writes y; bwd: reduce reads dy, x; elemt reads dy, x, writes dx
    tag = "syncbn_nhwc" if channels_last else "syncbn_nchw"
    return [dict(op=tag + "_fwd", us=fwd, bytes=3 * n, kernels="bn_local_stats + bn_combine + bn_elemt"),
            dict(op=tag + "_bwd", us=bwd, bytes=5 * n, kernels="bn_bwd_reduce + bn_bwd_elemt")]


def op_scale(iters):
    from apex.multi_tensor_apply import multi_tensor_applier
    from apex.multi_tensor_apply.ops import multi_tensor_scale

    sizes = [1024 * 1024] * 96 + [4096 * 1024] * 48 + [30528 * 1024]
    src = [torch.randn(s, device=DEV, dtype=torch.bfloat16) for s in sizes]
    dst = [torch.empty(s, device=DEV, dtype=torch.float32) for s in sizes]
    noop = torch.zeros(1, dtype=torch.int32, device=DEV)
    n = sum(sizes)
    us = _time(lambda: multi_tensor_applier(multi_tensor_scale, noop, [src, dst], 1.0 / 1024), iters)
    return [dict(op="multi_tensor_scale_bf16_to_fp32", us=us, bytes=n * 6, params=n, kernels="mt scale")]


OPS = dict(adam=op_adam, ln=op_ln, bdaln=op_bdaln, lamb=op_lamb, xent=op_xent, syncbn=op_syncbn,
           syncbn_nhwc=lambda it: op_syncbn(it, True), scale=op_scale)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default=",".join(OPS))
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    import apex._ext as e

    e.require()
    for name in args.ops.split(","):
        try:
            for r in OPS[name](args.iters):
                r["us"] = round(r["us"], 1)
                r["TBps_logical"] = round(r["bytes"] / r["us"] / 1e6, 3)
                print(json.dumps(r), flush=True)
        except Exception as ex:  # one op failing must not hide the others' numbers
            print(json.dumps({"op": name, "error": repr(ex)[:300]}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
