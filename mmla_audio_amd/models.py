"""``load_model(path).predict(x)`` facade for the two reference networks.

Replaces ``tf.keras.models.load_model`` + ``Model.predict`` at the reference call sites
(OD ``record_on_pc.py:88,159``; SI ``record_on_pc.py:77,136``;
``speaker_identification_post_processing.py:206,272``; ``overlap_detection_post_processing.py``).

Weights: if ``<path>/variables/variables.data-00000-of-00001`` exists the trained tensors are read
from the TF bundle (``tfbundle.load_bundle``).  The reference does not ship that file
(``.MISSING_LARGE_BLOBS``); like ``tf.keras.models.load_model`` on an incomplete SavedModel, loading
then raises -- a drop-in must not log confident labels from a random net.  Seeded synthetic
weights in the exact reference layout are used only on request (``allow_synthetic=True``;
``model.synthetic`` is then True).
"""
import os
import warnings

import numpy as np

from . import _lib, tfbundle, weights


def _layout_from_path(path):
    """(kind, n_classes, head) from the bundle index (tfbundle.layout), or None without one"""
    idx = os.path.join(path, 'variables', 'variables.index')
    if os.path.exists(idx):
        try:
            return tfbundle.layout(tfbundle.variable_shapes(idx))[:3]
        except ValueError:
            return None
    return None


def _kind_from_path(path):
    lay = _layout_from_path(path)
    if lay is not None:
        return lay[0]
    low = path.replace('\\', '/').lower()
    return weights.OD if 'overlap' in low or 'timit2' in low or 'timit1' in low else weights.SI


class _Model:
    kind = None

    def __init__(self, W, n_classes, head, device=None, synthetic=False):
        self.ctx = _lib.default_context(device) if device is None or isinstance(device, int) else device
        self.n_classes = n_classes
        self.head = head
        self.synthetic = synthetic
        self.W = W
        self.ctx.load_weights(self.kind, weights.pack(self.kind, W, n_classes), n_classes, head)

    def _ensure_loaded(self):
        # several models can share one context; re-load if another model of this kind replaced ours
        cls = self.ctx.od_classes if self.kind == weights.OD else self.ctx.si_classes
        if getattr(self.ctx, f'_owner_{self.kind}', None) is not self or cls != self.n_classes:
            self.ctx.load_weights(self.kind, weights.pack(self.kind, self.W, self.n_classes),
                                  self.n_classes, self.head)
            setattr(self.ctx, f'_owner_{self.kind}', self)


class OverlapDetectionModel(_Model):
    """OD-NET (ResLSTM, overlap_detector_temp.py:280-303): predict(float32 [N,128,151,3]) -> [N,2]."""
    kind = weights.OD

    def __init__(self, W, device=None, synthetic=False):
        super().__init__(W, 2, _lib.HEAD_SOFTMAX, device, synthetic)
        setattr(self.ctx, f'_owner_{self.kind}', self)

    def predict(self, x, batch_size=None, verbose=0):
        self._ensure_loaded()
        x = np.asarray(x)
        if x.ndim != 4 or x.shape[1:] != (128, 151, 3):
            raise ValueError(f'OD model expects [N,128,151,3], got {x.shape}')
        return self.ctx.od_forward(x)

    def predict_wavs(self, pcm, lens=None):
        """Fused WAV -> class (no PNG round trip): int16 [N, L] -> (probs [N,2], argmax [N]
        (-1 = 'silent', fewer than 4000 samples: record_on_pc.py:141-154), silent [N])."""
        self._ensure_loaded()
        return self.ctx.od_pipeline(pcm, lens)


class SpeakerIdModel(_Model):
    """SI-NET (res_model + head, speaker_identification.py:193-218,401-410): predict([N,256,39])."""
    kind = weights.SI

    def __init__(self, W, n_classes, head, device=None, synthetic=False):
        super().__init__(W, n_classes, head, device, synthetic)
        setattr(self.ctx, f'_owner_{self.kind}', self)

    def predict(self, x, batch_size=None, verbose=0):
        self._ensure_loaded()
        x = np.asarray(x)
        if x.ndim != 3 or x.shape[1:] != (256, 39):
            raise ValueError(f'SI model expects [N,256,39], got {x.shape}')
        return self.ctx.si_forward(x)

    def predict_wavs(self, pcm, lens=None):
        """Fused WAV -> speaker: -> (probs [N,K], argmax [N] (-1 = 'silent'), silent [N])."""
        self._ensure_loaded()
        return self.ctx.si_pipeline(pcm, lens)


def load_model(path, kind=None, n_classes=None, head=None, seed=0, device=None,
               allow_synthetic=False):
    """tf.keras.models.load_model drop-in for the reference's model directories: the OD base models
    (timit/models/timit{1.0,2.0}), the SI base model (timit/model, Dense(630) softmax) and the
    deployed SI model transfer_learning saves (experiment/model: the sliced base nested inside a
    model with the customized_dense sigmoid head, speaker_identification.py:401-410,456) -- the
    layout is read from the bundle index (tfbundle.layout), K and the head from its head kernel.
    Raises FileNotFoundError when the trained variables are absent, unless allow_synthetic=True."""
    lay = _layout_from_path(path)
    kind = (lay[0] if lay else _kind_from_path(path)) if kind is None else kind
    synthetic = False
    shard = os.path.join(path, 'variables', 'variables.data-00000-of-00001')
    if os.path.exists(shard):
        # present: any failure (a corrupt bundle, libmmla.so missing for the CRC) is a real error
        W, (bkind, bk, bhead) = tfbundle.load_bundle(path, with_layout=True)
        if bkind != kind:
            raise ValueError(f'{path}: bundle holds a {"OD" if bkind == weights.OD else "SI"} model')
        if kind == weights.SI:
            n_classes = bk
            head = bhead if head is None else head
    else:
        if not allow_synthetic:
            raise FileNotFoundError(
                f'{path}: trained variables not found ({shard} is absent); the reference ships only '
                f'variables.index (.MISSING_LARGE_BLOBS). Pass allow_synthetic=True for seeded '
                f'synthetic weights in the reference layout.')
        if lay is not None and kind == weights.SI:   # the layout the index names (K, head)
            n_classes = lay[1] if n_classes is None else n_classes
            head = lay[2] if head is None else head
        warnings.warn(f'{path}: trained weights absent (reference .MISSING_LARGE_BLOBS); using seeded '
                      f'synthetic weights in the reference layout (seed={seed})')
        W = weights.synthetic(kind, seed=seed, n_classes=n_classes)
        synthetic = True
    if kind == weights.OD:
        return OverlapDetectionModel(W, device=device, synthetic=synthetic)
    if n_classes is None:
        n_classes = W['layer_with_weights-42/kernel'].shape[1]
    if head is None:
        head = _lib.HEAD_SOFTMAX if n_classes == 630 else _lib.HEAD_SIGMOID
    return SpeakerIdModel(W, n_classes, head, device=device, synthetic=synthetic)
