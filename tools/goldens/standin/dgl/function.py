"""Stand-in for dgl.function: only the builtin `sum` reducer is needed."""


class _SumReducer:
    def __init__(self, msg, out):
        self.msg, self.out = msg, out


def sum(msg, out):  # noqa: A001 - mirrors dgl.function.sum
    return _SumReducer(msg, out)
