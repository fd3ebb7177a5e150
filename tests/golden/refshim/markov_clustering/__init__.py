"""Import-only stand-in (MCL is not on the measured path)."""

def run_mcl(*a, **k):
    raise NotImplementedError


def get_clusters(*a, **k):
    raise NotImplementedError
