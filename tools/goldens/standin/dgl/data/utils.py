"""Stand-in: the remote dataset helpers are never called offline."""


def _unavailable(*a, **k):
    raise RuntimeError("remote DGL datasets are unavailable in this container")


download = extract_archive = _unavailable


def get_download_dir():
    return "/nonexistent"


def _get_dgl_url(path):
    return "offline://" + path
