"""Placeholder until the C++ runtime is built (see native/__init__)."""


def available() -> bool:
    return False


def build():
    raise NotImplementedError("native runtime not yet available")
