"""mmla_audio_amd -- MI355X-native hot path of lizaibeim/mmla-audio.

WAV -> features -> network -> class for the OverlapDetection and SpeakerIdentification pipelines,
as hand-written gfx950 HIP kernels behind the C ABI in ``include/mmla.h`` (``libmmla.so``), bound
here with ctypes under the reference's own names:

  overlap_features_generator.OverlapFeaturesGenerator   (reference overlap_features_generator.py)
  speaker_identification.input_feature_gen / delta /
      make_feature_experiment                           (reference speaker_identification.py)
  models.load_model(path).predict(x) / .predict_wavs    (tf.keras.models.load_model)
  distributed.sharded_predict                           (1/2/4/8 GPUs, RCCL all-gather of logits)

Importing this package does not touch the GPU; the first call that needs it dlopens libmmla.so
and raises if it (or a HIP device) is missing -- there is no CPU fallback.
"""
from . import weights, tfbundle  # noqa: F401

__all__ = ['weights', 'tfbundle', 'load_model', 'OverlapFeaturesGenerator', 'input_feature_gen',
           'delta']


def __getattr__(name):
    if name == 'load_model':
        from .models import load_model
        return load_model
    if name == 'OverlapFeaturesGenerator':
        from .overlap_features_generator import OverlapFeaturesGenerator
        return OverlapFeaturesGenerator
    if name in ('input_feature_gen', 'delta', 'make_feature_experiment'):
        from . import speaker_identification
        return getattr(speaker_identification, name)
    raise AttributeError(name)
