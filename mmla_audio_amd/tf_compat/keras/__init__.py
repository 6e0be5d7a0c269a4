"""``tf.keras``: ``models.load_model`` (the reference's only Keras call on the hot path) and an
inert ``backend`` (imported as ``K`` by the reference scripts, never used on the path)."""
from . import backend, models  # noqa: F401
