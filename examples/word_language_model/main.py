"""Word-level RNN language model (Wikitext-2 format) with apex mixed precision.

Capabilities of reference examples/word_language_model/main.py (manual fp16, R-35) and
main_fp16_optimizer.py (R-36):
  --precision fp32 | manual (half model + fp32 master params, static loss scale)
              | fp16_opt (FP16_Optimizer, static or dynamic scale, clip_master_grads)
              | amp (amp.initialize O1 cast policy, or O2)
  --backend torch (nn.LSTM on MIOpen) | apex (apex.RNN fused cells)
Without --data files a synthetic corpus is generated (no downloads here).

  python examples/word_language_model/main.py --epochs 6 --precision fp16_opt --dynamic-loss-scale --tied
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import tempfile
import time

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import data  # noqa: E402
from model import RNNModel, repackage_hidden  # noqa: E402

from apex import amp  # noqa: E402
from apex.fp16_utils import (FP16_Optimizer, master_params_to_model_params,  # noqa: E402
                             model_grads_to_master_grads, prep_param_lists)


def parse(argv=None):
    p = argparse.ArgumentParser(description="RNN/LSTM language model with apex")
    p.add_argument("--data", default="", help="dir with train/valid/test.txt (synthetic if empty)")
    p.add_argument("--model", default="LSTM", choices=["LSTM", "GRU", "RNN_TANH", "RNN_RELU"])
    p.add_argument("--backend", default="torch", choices=["torch", "apex"])
    p.add_argument("--emsize", type=int, default=200)
    p.add_argument("--nhid", type=int, default=200)
    p.add_argument("--nlayers", type=int, default=2)
    p.add_argument("--lr", type=float, default=20)
    p.add_argument("--clip", type=float, default=0.25)
    p.add_argument("--epochs", type=int, default=6)
    p.add_argument("--batch_size", type=int, default=20)
    p.add_argument("--bptt", type=int, default=35)
    p.add_argument("--dropout", type=float, default=0.2)
    p.add_argument("--tied", action="store_true")
    p.add_argument("--seed", type=int, default=1111)
    p.add_argument("--log-interval", type=int, default=200)
    p.add_argument("--save", default=os.path.join(tempfile.gettempdir(), "wlm_model.pt"))
    p.add_argument("--precision", default="fp32", choices=["fp32", "manual", "fp16_opt", "amp"])
    p.add_argument("--half-dtype", default="fp16", choices=["fp16", "bf16"])
    p.add_argument("--opt-level", default="O1")
    p.add_argument("--static-loss-scale", type=float, default=1.0)
    p.add_argument("--dynamic-loss-scale", action="store_true")
    p.add_argument("--max-batches", type=int, default=0, help="cap batches per epoch (smoke runs)")
    return p.parse_args(argv)


def batchify(d, bsz, device):
    nb = d.size(0) // bsz
    return d[: nb * bsz].view(bsz, -1).t().contiguous().to(device)


def get_batch(source, i, bptt):
    n = min(bptt, len(source) - 1 - i)
    return source[i:i + n], source[i + 1:i + 1 + n].reshape(-1)


def main(argv=None):
    args = parse(argv)
    torch.manual_seed(args.seed)
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    half = torch.float16 if (args.half_dtype == "fp16" and dev.type == "cuda") else torch.bfloat16
    path = args.data or data.synthetic_corpus(os.path.join(tempfile.gettempdir(), "apex_wlm_synth"))
    corpus = data.Corpus(path)
    train_data = batchify(corpus.train, args.batch_size, dev)
    val_data = batchify(corpus.valid, 10, dev)
    test_data = batchify(corpus.test, 10, dev)
    ntokens = len(corpus.dictionary)
    model = RNNModel(args.model, ntokens, args.emsize, args.nhid, args.nlayers, args.dropout, args.tied,
                     args.backend).to(dev)
    criterion = nn.CrossEntropyLoss()
    opt = None
    master = None
    if args.precision in ("manual", "fp16_opt"):
        model = model.to(half)
    if args.precision == "manual":
        model_params, master = prep_param_lists(model)
    elif args.precision == "fp16_opt":
        opt = FP16_Optimizer(torch.optim.SGD(model.parameters(), lr=args.lr), static_loss_scale=args.static_loss_scale,
                             dynamic_loss_scale=args.dynamic_loss_scale, verbose=False)
    elif args.precision == "amp":
        opt = torch.optim.SGD(model.parameters(), lr=args.lr)
        model, opt = amp.initialize(model, opt, opt_level=args.opt_level, half_dtype=half,
                                    loss_scale="dynamic" if args.dynamic_loss_scale else args.static_loss_scale,
                                    verbosity=0)
    lr = args.lr

    def evaluate(source):
        model.eval()
        total, n = 0.0, 0
        hidden = model.init_hidden(10)
        with torch.no_grad():
            for i in range(0, source.size(0) - 1, args.bptt):
                x, y = get_batch(source, i, args.bptt)
                out, hidden = model(x, hidden)
                total += len(x) * criterion(out.view(-1, ntokens).float(), y).item()
                n += len(x)
                hidden = repackage_hidden(hidden, model)
        return total / max(n, 1)

    def train(epoch):
        nonlocal lr
        model.train()
        total, start = 0.0, time.time()
        hidden = model.init_hidden(args.batch_size)
        for batch, i in enumerate(range(0, train_data.size(0) - 1, args.bptt)):
            if args.max_batches and batch >= args.max_batches:
                break
            x, y = get_batch(train_data, i, args.bptt)
            hidden = repackage_hidden(hidden, model)
            out, hidden = model(x, hidden)
            loss = criterion(out.view(-1, ntokens).float(), y)
            if args.precision == "manual":
                model.zero_grad()
                (loss * args.static_loss_scale).backward()
                model_grads_to_master_grads(model_params, master)
                for p in master:
                    p.grad.data.mul_(1.0 / args.static_loss_scale)
                torch.nn.utils.clip_grad_norm_(master, args.clip)
                for p in master:
                    p.data.add_(p.grad.data, alpha=-lr)
                master_params_to_model_params(model_params, master)
            elif args.precision == "fp16_opt":
                opt.zero_grad()
                opt.backward(loss)
                opt.clip_master_grads(args.clip)
                for g in opt.param_groups:
                    g["lr"] = lr
                opt.step()
            elif args.precision == "amp":
                opt.zero_grad()
                with amp.scale_loss(loss, opt) as sl:
                    sl.backward()
                torch.nn.utils.clip_grad_norm_(amp.master_params(opt), args.clip)
                for g in opt.param_groups:
                    g["lr"] = lr
                opt.step()
            else:
                model.zero_grad()
                loss.backward()
                torch.nn.utils.clip_grad_norm_(model.parameters(), args.clip)
                with torch.no_grad():
                    for p in model.parameters():
                        p.add_(p.grad, alpha=-lr)
            total += loss.item()
            if batch % args.log_interval == 0 and batch > 0:
                cur = total / args.log_interval
                ms = (time.time() - start) * 1000 / args.log_interval
                print("| epoch {:3d} | {:5d} batches | lr {:02.2f} | ms/batch {:5.2f} | loss {:5.2f} | ppl {:8.2f}"
                      .format(epoch, batch, lr, ms, cur, math.exp(min(cur, 50))), flush=True)
                total, start = 0.0, time.time()

    best = None
    for epoch in range(1, args.epochs + 1):
        t0 = time.time()
        train(epoch)
        val = evaluate(val_data)
        print("| end of epoch {:3d} | time {:5.2f}s | valid loss {:5.2f} | valid ppl {:8.2f}"
              .format(epoch, time.time() - t0, val, math.exp(min(val, 50))), flush=True)
        if best is None or val < best:
            torch.save({"model": model.state_dict(), "args": vars(args), "vocab": corpus.dictionary.idx2word},
                       args.save)
            best = val
        else:
            lr /= 4.0
    ck = torch.load(args.save, weights_only=True)
    model.load_state_dict(ck["model"])
    test = evaluate(test_data)
    print("| End of training | test loss {:5.2f} | test ppl {:8.2f}".format(test, math.exp(min(test, 50))))
    return test


if __name__ == "__main__":
    main()
