"""Clustering (reference ``heat/cluster``): KMeans, KMedians, KMedoids, Spectral."""
from ._kcluster import _KCluster
from .kmeans import KMeans
from .kmedians import KMedians
from .kmedoids import KMedoids
from .spectral import Spectral

__all__ = ["KMeans", "KMedians", "KMedoids", "Spectral"]
