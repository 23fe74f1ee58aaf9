from .brax import Brax
from .gym import Gym, CapEpisode, Normalizer
from .env_pool import EnvPool
from .envs import get_environment, Ant, CartPole, Pendulum, MountainCarContinuous
