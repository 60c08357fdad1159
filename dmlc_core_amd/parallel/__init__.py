"""Distributed launch, rendezvous (dmlc tracker) and RCCL collectives."""
from __future__ import annotations

__all__ = []
