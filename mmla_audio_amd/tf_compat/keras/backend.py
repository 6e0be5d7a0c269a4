"""``tensorflow.keras.backend``: the reference scripts import it as ``K`` (OD ``record_on_pc.py:19``,
``overlap_detection_post_processing.py:15``, SI ``record_on_pc.py:19``) and use nothing from it on
the hot path."""


def clear_session():
    """Keras frees its graph state here; the GPU contexts hold no per-session graph."""


def floatx():
    return 'float32'
