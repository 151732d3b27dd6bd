# User line transform hook (reference: bin/transform.py, executed by Jython there; plain
# CPython here). transform(raw_bytes) -> list of ytk-format lines; return [] to drop a line.
# Example: libsvm "label f:v f:v" -> "1###label###f:v,f:v".


def transform(bytesarr):
    line = bytesarr.decode("utf-8")
    cols = line.split(" ")
    return ["###".join(["1", cols[0], ",".join(cols[1:])])]
