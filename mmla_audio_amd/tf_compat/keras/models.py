"""``tf.keras.models`` for OD ``record_on_pc.py:88``, ``overlap_detection_post_processing.py:154``,
SI ``record_on_pc.py:77`` and ``speaker_identification_post_processing.py:206``."""
from ... import models as _models


def load_model(filepath, custom_objects=None, compile=True, options=None):
    """``tf.keras.models.load_model(filepath)`` -> the OD / SI model of that SavedModel directory,
    predicting on the GPU (``mmla_audio_amd.models.load_model``: trained variables from
    ``variables/variables.{index,data-*}``; FileNotFoundError if the data shard is absent, as TF
    fails on an incomplete SavedModel).  ``custom_objects`` / ``compile`` / ``options`` are accepted
    and ignored: inference needs no compiled training state."""
    return _models.load_model(str(filepath))
