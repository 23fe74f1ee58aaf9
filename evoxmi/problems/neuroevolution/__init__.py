"""Neuroevolution problems (reference ``problems/neuroevolution``)."""
from .reinforcement_learning import Brax, CapEpisode, EnvPool, Gym, get_environment
from .supervised_learning import TensorflowDataset
