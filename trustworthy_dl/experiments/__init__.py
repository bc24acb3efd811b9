"""Experiment runner (reference experiment_runner.py)."""
from .runner import ExperimentConfig, ExperimentRunner, main  # noqa: F401
