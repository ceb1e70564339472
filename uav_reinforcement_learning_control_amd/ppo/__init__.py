from .gae import gae
from .policy import ActorCritic
from .ppo import PPO, PPOConfig, allreduce_mean_, ppo_loss

__all__ = ["gae", "ActorCritic", "PPO", "PPOConfig", "ppo_loss", "allreduce_mean_"]
