"""The examples/ demos run end to end on 2 CPU ranks through the launcher."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("script,args,expect", [
    ("examples/cluster/demo_kclustering.py", [], "clusters recovered exactly: True"),
    ("examples/classification/demo_knn.py", [], "fold accuracies"),
    ("examples/lasso/demo.py", [], "lambda="),
    ("examples/nn/mnist.py", ["--epochs", "1", "--samples", "512"], "epoch 0"),
    ("examples/nn/imagenet.py", ["--epochs", "2", "--samples", "256", "--batch-size", "16", "--image-size", "32",
                                 "--width", "8", "--classes", "10", "--layers", "1,1"], '"example": "imagenet"'),
    ("examples/nn/imagenet-DASO.py", ["--epochs", "3", "--samples", "256", "--batch-size", "16", "--image-size",
                                      "32", "--width", "8", "--classes", "10", "--layers", "1,1"],
     '"example": "imagenet-DASO"'),
])
def test_example(script, args, expect):
    env = dict(os.environ, HEAT_COMM_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    res = subprocess.run([sys.executable, "-m", "heat_amd.run", "-n", "2", "--backend", "gloo",
                          os.path.join(REPO, script)] + args, cwd=REPO, env=env, capture_output=True, text=True,
                         timeout=600)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert expect in res.stdout


def test_datasets():
    import numpy as np
    import heat_amd as ht

    X, y = ht.datasets.iris()
    assert X.shape == (150, 4) and y.shape == (150,)
    assert np.bincount(y.numpy()).tolist() == [50, 50, 50]
    km = ht.cluster.KMeans(n_clusters=3, init="kmeans++", random_state=1).fit(X)
    assert km.cluster_centers_.shape == (3, 4)
    Xd, yd = ht.datasets.diabetes()
    assert Xd.shape == (442, 10) and yd.shape == (442, 1)
