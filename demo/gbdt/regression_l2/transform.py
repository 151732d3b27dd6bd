"""Line transform hook for the exact-greedy GBDT demo: a raw LibSVM line
``label idx:val idx:val ...`` becomes the ytk-learn line ``1###label###idx:val,...``
(weight 1). Same contract as bin/transform.py: bytes in, list of lines out ([] drops it)."""


def transform(raw: bytes):
    parts = raw.decode("utf-8").strip().split()
    if not parts:
        return []
    return ["###".join(["1", parts[0], ",".join(parts[1:])])]
