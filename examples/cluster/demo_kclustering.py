"""
k-clustering demo (reference ``examples/cluster/demo_kClustering.py``): KMeans, KMedians and
KMedoids on four well separated spherical clusters, distributed along the samples.

    python -m heat_amd.run -n 4 examples/cluster/demo_kclustering.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import heat_amd as ht  # noqa: E402


def main():
    centers = [[4.0, 4.0, 4.0], [-4.0, -4.0, -4.0], [4.0, -4.0, 4.0], [-4.0, 4.0, -4.0]]
    data, truth = ht.datasets.make_blobs(4000, centers, std=1.0, seed=1, split=0)
    for cls in (ht.cluster.KMeans, ht.cluster.KMedians, ht.cluster.KMedoids):
        est = cls(n_clusters=4, init="kmeans++", random_state=3)
        labels = est.fit_predict(data)
        c = est.cluster_centers_
        if ht.MPI_WORLD.rank == 0:
            print("{}: centers\n{}".format(cls.__name__, c.numpy().round(2)))
        # purity: every true cluster maps to one label
        lab, tru = labels.numpy().ravel(), truth.numpy().ravel()
        if ht.MPI_WORLD.rank == 0:
            pure = all(len(set(lab[tru == t])) == 1 for t in range(4))
            print("  clusters recovered exactly: {}".format(pure))


if __name__ == "__main__":
    main()
