"""Utilities: .ot checkpoints, labels, dataset layout, latency statistics."""
