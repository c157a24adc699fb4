"""Utilities: synthetic workloads, logging/metrics, config, auth helpers."""
