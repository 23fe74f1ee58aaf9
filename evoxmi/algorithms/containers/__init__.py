"""Algorithm containers (reference ``algorithms/containers/``): cooperative
co-evolution, clustered / randomly-masked decomposition, per-leaf tree algorithms, and
batched independent runs (vmap)."""
from .batched import BatchedRuns
from .coevolution import Coevolution, VectorizedCoevolution
from .clustered_algorithm import ClusterdAlgorithm, ClusteredAlgorithm, RandomMaskAlgorithm
from .tree_algorithm import FlattenParam, TreeAlgorithm
