"""Test-only stub: QuantileTree is out of scope."""


class QuantileTree:

    def __init__(self, *args, **kwargs):
        raise NotImplementedError("QuantileTree is out of scope")
