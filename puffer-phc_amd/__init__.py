"""puffer_phc_amd — MI355X-native PHC imitation rollout + PPO hot path."""
