"""Sample text from a checkpoint written by main.py (capability of reference
examples/word_language_model/generate.py). Checkpoint loads with weights_only=True.

  python examples/word_language_model/generate.py --checkpoint /tmp/wlm_model.pt --words 200
"""
import argparse
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from model import RNNModel  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--checkpoint", default=os.path.join(tempfile.gettempdir(), "wlm_model.pt"))
    p.add_argument("--outf", default="generated.txt")
    p.add_argument("--words", type=int, default=1000)
    p.add_argument("--seed", type=int, default=1111)
    p.add_argument("--temperature", type=float, default=1.0)
    p.add_argument("--log-interval", type=int, default=100)
    args = p.parse_args(argv)
    if args.temperature < 1e-3:
        p.error("--temperature has to be greater or equal 1e-3")
    torch.manual_seed(args.seed)
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    ck = torch.load(args.checkpoint, map_location="cpu", weights_only=True)
    a, vocab = ck["args"], ck["vocab"]
    model = RNNModel(a["model"], len(vocab), a["emsize"], a["nhid"], a["nlayers"], 0.0, a["tied"], a["backend"])
    dt = next(iter(ck["model"].values())).dtype
    model = model.to(dev, dt)
    model.load_state_dict(ck["model"])
    model.eval()
    hidden = model.init_hidden(1)
    x = torch.randint(len(vocab), (1, 1), dtype=torch.long, device=dev)
    words = []
    with torch.no_grad():
        for i in range(args.words):
            out, hidden = model(x, hidden)
            weights = out.squeeze().float().div(args.temperature).exp()
            idx = torch.multinomial(weights, 1)[0]
            x.fill_(idx)
            words.append(vocab[idx])
            if i % args.log_interval == 0:
                print("| Generated {}/{} words".format(i, args.words))
    with open(args.outf, "w") as f:
        for i, w in enumerate(words):
            f.write(w + ("\n" if i % 20 == 19 else " "))
    return words


if __name__ == "__main__":
    main()
