"""Word-level corpus for the language-model example.

Reads ``train.txt`` / ``valid.txt`` / ``test.txt`` (one sentence per line, whitespace tokens,
``<eos>`` appended per line) from ``--data``. Without files (no dataset can be downloaded
here), ``synthetic_corpus`` writes a Zipf-distributed bigram text of the same format so the
example runs end to end."""
from __future__ import annotations

import os

import torch


class Dictionary:
    def __init__(self):
        self.word2idx = {}
        self.idx2word = []

    def add_word(self, word):
        idx = self.word2idx.get(word)
        if idx is None:
            idx = self.word2idx[word] = len(self.idx2word)
            self.idx2word.append(word)
        return idx

    def __len__(self):
        return len(self.idx2word)


class Corpus:
    def __init__(self, path):
        self.dictionary = Dictionary()
        self.train = self.tokenize(os.path.join(path, "train.txt"))
        self.valid = self.tokenize(os.path.join(path, "valid.txt"))
        self.test = self.tokenize(os.path.join(path, "test.txt"))

    def tokenize(self, path):
        """One pass: grow the dictionary and collect ids."""
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        ids = []
        add = self.dictionary.add_word
        with open(path, "r", encoding="utf-8") as f:
            for line in f:
                ids.extend(add(w) for w in line.split() + ["<eos>"])
        return torch.tensor(ids, dtype=torch.int64)


def synthetic_corpus(path, vocab=2000, lines=(4000, 400, 400), seed=0):
    """Write a learnable synthetic corpus (Zipf unigrams + a fixed successor per word)."""
    os.makedirs(path, exist_ok=True)
    g = torch.Generator().manual_seed(seed)
    probs = 1.0 / torch.arange(1, vocab + 1, dtype=torch.float64)
    succ = torch.randint(0, vocab, (vocab,), generator=g)
    for name, n in zip(("train", "valid", "test"), lines):
        with open(os.path.join(path, name + ".txt"), "w") as f:
            for _ in range(n):
                L = int(torch.randint(5, 20, (1,), generator=g))
                w = int(torch.multinomial(probs, 1, generator=g))
                words = []
                for _ in range(L):
                    words.append("w%d" % w)
                    w = int(succ[w]) if torch.rand(1, generator=g) < 0.7 else int(torch.multinomial(probs, 1,
                                                                                                  generator=g))
                f.write(" ".join(words) + "\n")
    return path
