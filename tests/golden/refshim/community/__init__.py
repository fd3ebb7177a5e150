"""Import-only stand-in for python-louvain."""

def best_partition(*a, **k):
    raise NotImplementedError
