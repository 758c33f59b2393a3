"""``CryptoAlgorithm`` -- same contract as quantum_resistant_p2p/crypto/algorithm_base.py:8-57.

name (abstract), display_name (defaults to name), description (abstract),
is_using_mock (always False), actual_variant (self.variant or None), and
get_security_info() with keys name / mock_implementation / description
[/ actual_variant] [/ security_level].
"""
from __future__ import annotations

import abc
from typing import Optional


class CryptoAlgorithm(abc.ABC):
    @property
    @abc.abstractmethod
    def name(self) -> str:
        ...

    @property
    def display_name(self) -> str:
        return self.name

    @property
    @abc.abstractmethod
    def description(self) -> str:
        ...

    @property
    def is_using_mock(self) -> bool:
        return False

    @property
    def actual_variant(self) -> Optional[str]:
        return getattr(self, "variant", None) or None

    def get_security_info(self) -> dict:
        info = {
            "name": self.display_name,
            "mock_implementation": False,
            "description": self.description,
        }
        if self.actual_variant:
            info["actual_variant"] = self.actual_variant
        if hasattr(self, "security_level"):
            info["security_level"] = self.security_level
        return info
