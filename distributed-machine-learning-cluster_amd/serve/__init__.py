"""Serving: local cluster launcher/driver for the C++ ``dmlc-node`` binary
(membership, SDFS, predict jobs) — see ``cluster.py``."""
