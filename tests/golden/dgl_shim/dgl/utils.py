"""Restated DGL 2.1.0 ``dgl.utils.expand_as_pair`` for non-block graphs; test-only."""


def expand_as_pair(input_, g=None):
    if isinstance(input_, tuple):
        return input_
    return input_, input_
