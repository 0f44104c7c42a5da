"""
kNN demo (reference ``examples/classification/demo_knn.py``): k-fold style evaluation of
``KNeighborsClassifier`` on the (synthetic) iris data.

    python -m heat_amd.run -n 2 examples/classification/demo_knn.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

import heat_amd as ht  # noqa: E402


def main():
    X, y = ht.datasets.iris(split=0)
    Xn, yn = X.numpy(), y.numpy()
    rng = np.random.default_rng(0)
    perm = rng.permutation(len(yn))
    folds = np.array_split(perm, 5)
    accs = []
    for i, test in enumerate(folds):
        train = np.concatenate([f for j, f in enumerate(folds) if j != i])
        knn = ht.classification.KNeighborsClassifier(n_neighbors=5)
        knn.fit(ht.array(Xn[train], split=0), ht.array(yn[train], split=0))
        pred = knn.predict(ht.array(Xn[test], split=0)).numpy().ravel()
        accs.append(float((pred == yn[test]).mean()))
    if ht.MPI_WORLD.rank == 0:
        print("fold accuracies:", [round(a, 3) for a in accs], "mean", round(float(np.mean(accs)), 3))


if __name__ == "__main__":
    main()
