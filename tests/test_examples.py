"""Smoke-run every example on CPU with tiny settings (subprocess, PYTHONPATH=repo)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")


def _run(args, tmp_path, torchrun=0, timeout=600):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    cmd = [sys.executable]
    if torchrun:
        cmd += ["-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
                "--nproc-per-node", str(torchrun)]
    r = subprocess.run(cmd + args, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("name", ["minimal.py", "closure.py", "save_load.py"])
def test_fp16_optimizer_simple(name, tmp_path):
    out = _run([os.path.join(EX, "FP16_Optimizer_simple", name), "--steps", "10"], tmp_path)
    assert "final loss" in out
    if name == "save_load.py":
        assert "identical params: True" in out


@pytest.mark.parametrize("torch_ddp", [False, True])
def test_fp16_optimizer_simple_distributed(tmp_path, torch_ddp):
    out = _run([os.path.join(EX, "FP16_Optimizer_simple", "distributed", "distributed_data_parallel.py"),
                "--steps", "5"] + (["--torch-ddp"] if torch_ddp else []), tmp_path, torchrun=2)
    assert out.count("final loss") == 2


IMNET = ["-a", "resnet18", "--image-size", "32", "-b", "4", "--train-size", "16", "--val-size", "8",
         "--num-classes", "10", "-j", "0", "-p", "2"]


@pytest.mark.parametrize("prec", ["fp32", "manual", "fp16_opt", "amp"])
def test_imagenet(prec, tmp_path):
    out = _run([os.path.join(EX, "imagenet", "main.py"), "--precision", prec, "--checkpoint",
                str(tmp_path / "ck.pt")] + IMNET, tmp_path)
    assert "Prec@1" in out
    out = _run([os.path.join(EX, "imagenet", "main.py"), "--precision", prec, "--checkpoint", str(tmp_path / "ck.pt"),
                "--resume", str(tmp_path / "ck.pt"), "--epochs", "2"] + IMNET, tmp_path)
    assert "Epoch [1]" in out


def test_imagenet_reducer_syncbn_distributed(tmp_path):
    out = _run([os.path.join(EX, "imagenet", "main_reducer.py"), "--sync-bn", "--checkpoint",
                str(tmp_path / "ck.pt")] + IMNET, tmp_path, torchrun=2)
    assert "Prec@1" in out


@pytest.mark.parametrize("prec,backend", [("fp32", "torch"), ("fp16_opt", "torch"), ("manual", "torch"),
                                          ("fp32", "apex")])
def test_word_language_model(prec, backend, tmp_path):
    ck = str(tmp_path / "wlm.pt")
    out = _run([os.path.join(EX, "word_language_model", "main.py"), "--epochs", "1", "--max-batches", "8",
                "--precision", prec, "--backend", backend, "--save", ck, "--nhid", "64", "--emsize", "64"], tmp_path)
    assert "test ppl" in out
    _run([os.path.join(EX, "word_language_model", "generate.py"), "--checkpoint", ck, "--words", "20"], tmp_path)
    assert (tmp_path / "generated.txt").exists()


def test_distributed_mnist(tmp_path):
    out = _run([os.path.join(EX, "distributed", "main.py"), "--epochs", "1", "--train-size", "512"], tmp_path,
               torchrun=2)
    assert "Accuracy" in out
