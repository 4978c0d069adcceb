"""Builtin reducer descriptors (restated DGL 2.1.0 ``dgl.function``); test-only."""


class _Reducer:
    def __init__(self, name, msg_field, out_field):
        self.name = name
        self.msg_field = msg_field
        self.out_field = out_field


def sum(msg, out):  # noqa: A001 - mirrors DGL's name
    return _Reducer("sum", msg, out)


def mean(msg, out):
    return _Reducer("mean", msg, out)


def max(msg, out):  # noqa: A001
    return _Reducer("max", msg, out)
