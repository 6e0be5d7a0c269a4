"""The reference's hot-path call-site statements that reach TensorFlow, as the statement text the
drop-in tests execute against ``mmla_audio_amd.tf_compat`` ("executes the reference's own
lines verbatim").  Each entry is (reference file, first line, statements); the CPU test
``test_tf_compat_cpu.py::test_call_site_text_matches_reference`` checks the text against
``/root/reference`` when it is present, so these are the reference's lines, dedented, and nothing
else.  They are a few API calls, the interface under test -- not a reference source file."""

OD_REALTIME = ('OverlapDetection/scripts/record_on_pc.py', 156, """\
image = tf.io.read_file(features_image_path2)
features_data = [tf.image.decode_png(image, 3)]
_input = tf.stack(features_data, axis=0).numpy().astype('float32')
prob = model.predict(_input)
key = str(np.argmax(prob, axis=1)[0])
""")

OD_OFFLINE = ('OverlapDetection/scripts/overlap_detection_post_processing.py', 204, """\
image = tf.io.read_file(features_image_path)
features_data = [tf.image.decode_png(image, 3)]
_input = tf.stack(features_data, axis=0).numpy().astype('float32')

prob = model.predict(_input)
""")

OD_LOAD = ('OverlapDetection/scripts/record_on_pc.py', 88, """\
model = tf.keras.models.load_model(model_path)
""")

OD_OFFLINE_LOAD = ('OverlapDetection/scripts/overlap_detection_post_processing.py', 154, """\
model = tf.keras.models.load_model(model_path)
""")

SI_LOAD = ('SpeakerIdentification/scripts/record_on_pc.py', 77, """\
model = tf.keras.models.load_model(model_path)
""")

SI_REALTIME = ('SpeakerIdentification/scripts/record_on_pc.py', 136, """\
prob = model.predict(x)
key = str(np.argmax(prob, axis=1)[0])
""")

SI_OFFLINE_LOAD = ('SpeakerIdentification/scripts/speaker_identification_post_processing.py', 206, """\
model = tf.keras.models.load_model(model_path)
""")

SI_OFFLINE = ('SpeakerIdentification/scripts/speaker_identification_post_processing.py', 272, """\
results = model.predict(test_x)
""")

ALL = (OD_REALTIME, OD_OFFLINE, OD_LOAD, OD_OFFLINE_LOAD, SI_LOAD, SI_REALTIME, SI_OFFLINE_LOAD,
       SI_OFFLINE)


def run(site, **names):
    """Execute a call site's statements with ``names`` bound (tf, np, model, paths ...); -> the
    namespace after execution."""
    ns = dict(names)
    exec(compile(site[2], f'{site[0]}:{site[1]}', 'exec'), ns)
    return ns
