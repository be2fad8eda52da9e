"""PPO on the device vector env: agents, GAE kernel, the update."""
