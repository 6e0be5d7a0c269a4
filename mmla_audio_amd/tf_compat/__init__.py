"""``import tensorflow as tf`` for the reference's hot-path call sites, on the MI355X path.

Every reference caller reaches the model and the decoded feature image through the ``tf`` name:

* OD ``record_on_pc.py:88,156-159`` and ``overlap_detection_post_processing.py:154,204-208``::

      model = tf.keras.models.load_model(model_path)
      image = tf.io.read_file(features_image_path2)
      features_data = [tf.image.decode_png(image, 3)]
      _input = tf.stack(features_data, axis=0).numpy().astype('float32')
      prob = model.predict(_input)

* SI ``record_on_pc.py:77,136`` and ``speaker_identification_post_processing.py:206,272``:
  ``tf.keras.models.load_model`` + ``model.predict``.

Switching a script changes its TensorFlow import lines only::

    -import tensorflow as tf
    -from tensorflow.keras import backend as K
    +from mmla_audio_amd import tf_compat as tf
    +from mmla_audio_amd.tf_compat.keras import backend as K

and every line below them runs unchanged: ``tf.keras.models.load_model`` returns
``mmla_audio_amd.models.load_model``'s model (its ``predict`` runs OD-NET / SI-NET on the GPU),
``tf.io.read_file`` / ``tf.image.decode_png`` decode the PNG ``generate_zcr_image`` wrote (zlib +
``mmla_png_unfilter``), and ``tf.stack(...).numpy()`` gives the ndarray ``predict`` takes.  This
is not TensorFlow: only what those call sites use exists, and anything else raises
AttributeError rather than running something different.
"""
import numpy as np



uint8 = np.dtype(np.uint8)
uint16 = np.dtype(np.uint16)
int32 = np.dtype(np.int32)
int64 = np.dtype(np.int64)
float32 = np.dtype(np.float32)
float64 = np.dtype(np.float64)
string = np.dtype(object)


class Tensor:
    """An eager tensor: an ndarray (or, for ``tf.io.read_file``, one bytes string) with
    ``.numpy()``, ``.shape`` and ``.dtype`` as the call sites use them."""

    __slots__ = ('_v',)

    def __init__(self, value):
        self._v = value

    def numpy(self):
        return self._v

    @property
    def shape(self):
        return () if isinstance(self._v, bytes) else self._v.shape

    @property
    def dtype(self):
        return string if isinstance(self._v, bytes) else self._v.dtype

    def __array__(self, dtype=None, copy=None):
        if isinstance(self._v, bytes):
            raise TypeError('a string tensor has no numeric array form')
        a = self._v
        return a if dtype is None else a.astype(dtype)

    def __len__(self):
        return len(self._v)

    def __getitem__(self, k):
        return Tensor(self._v[k])

    def __repr__(self):
        return f'<tf_compat.Tensor shape={self.shape} dtype={self.dtype}>'


def _value(x):
    return x.numpy() if isinstance(x, Tensor) else x


def convert_to_tensor(value, dtype=None):
    if isinstance(value, Tensor) and dtype is None:
        return value
    v = _value(value)
    if isinstance(v, (bytes, str)):
        return Tensor(v.encode() if isinstance(v, str) else v)
    return Tensor(np.asarray(v, dtype=dtype))


constant = convert_to_tensor


def stack(values, axis=0, name='stack'):
    """``tf.stack``: the tensors (same shape) joined along a new ``axis``."""
    arrs = [np.asarray(_value(v)) for v in values]
    if not arrs:
        raise ValueError('tf.stack needs at least one tensor')
    return Tensor(np.stack(arrs, axis=axis))


def cast(x, dtype, name=None):
    return Tensor(np.asarray(_value(x)).astype(dtype))


from . import image, io, keras  # noqa: E402,F401  (tf.image / tf.io / tf.keras; need Tensor above)
