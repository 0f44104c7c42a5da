"""The examples/ demos end to end on the GPU: one rank on cuda:0 (default device "gpu", the native
kernels) and two ranks sharing the card over gloo with device buffers, through the launcher
(``python -m heat_amd.run``, child processes only)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    ("examples/cluster/demo_kclustering.py", [], "clusters recovered exactly: True"),
    ("examples/classification/demo_knn.py", [], "fold accuracies"),
    ("examples/lasso/demo.py", [], "lambda="),
    ("examples/nn/mnist.py", ["--epochs", "1", "--samples", "512"], "epoch 0"),
    ("examples/nn/imagenet.py", ["--epochs", "2", "--samples", "256", "--batch-size", "16", "--image-size", "32",
                                 "--width", "8", "--classes", "10", "--layers", "1,1"], '"example": "imagenet"'),
    ("examples/nn/imagenet-DASO.py", ["--epochs", "3", "--samples", "256", "--batch-size", "16", "--image-size",
                                      "32", "--width", "8", "--classes", "10", "--layers", "1,1"],
     '"example": "imagenet-DASO"'),
]


@pytest.mark.parametrize("nprocs", [1, 2])
@pytest.mark.parametrize("script,args,expect", CASES)
def test_example_on_gpu(script, args, expect, nprocs):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, HEAT_AMD_DEFAULT_DEVICE="gpu", HEAT_COMM_TIMEOUT="60")
    cmd = [sys.executable, "-m", "heat_amd.run", "-n", str(nprocs)]
    if nprocs > 1:
        cmd += ["--backend", "gloo"]   # RCCL refuses two ranks on one device
        env["HEAT_COMM_BACKEND"] = "gloo"
    res = subprocess.run(cmd + [os.path.join(REPO, script)] + args, cwd=REPO, env=env, capture_output=True, text=True,
                         timeout=280)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert expect in res.stdout
