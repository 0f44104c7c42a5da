"""
Model zoo index: every estimator / trainable model family of the framework in one namespace,
with a registry for programmatic discovery (``heat_amd.models.REGISTRY``).
"""
from ..cluster import KMeans, KMedians, KMedoids, Spectral
from ..regression import Lasso
from ..naive_bayes import GaussianNB
from ..classification import KNeighborsClassifier
from ..graph import Laplacian
from ..nn import DataParallel, DataParallelMultiGPU
from ..optim import DASO, DataParallelOptimizer

REGISTRY = {
    "kmeans": KMeans,
    "kmedians": KMedians,
    "kmedoids": KMedoids,
    "spectral": Spectral,
    "lasso": Lasso,
    "gaussian_nb": GaussianNB,
    "knn": KNeighborsClassifier,
}

__all__ = ["KMeans", "KMedians", "KMedoids", "Spectral", "Lasso", "GaussianNB", "KNeighborsClassifier", "Laplacian",
           "DataParallel", "DataParallelMultiGPU", "DASO", "DataParallelOptimizer", "REGISTRY"]
