"""``tf.io`` for ``record_on_pc.py:156`` / ``overlap_detection_post_processing.py:204``."""


def read_file(filename, name=None):
    """``tf.io.read_file``: the file's bytes as a scalar string tensor."""
    from . import Tensor, _value
    path = _value(filename)
    if isinstance(path, bytes):
        path = path.decode()
    with open(path, 'rb') as f:
        return Tensor(f.read())


def write_file(filename, contents, name=None):
    from . import _value
    path = _value(filename)
    data = _value(contents)
    with open(path.decode() if isinstance(path, bytes) else path, 'wb') as f:
        f.write(data.encode() if isinstance(data, str) else bytes(data))
