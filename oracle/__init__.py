"""CPU oracle for the mmla-audio hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, in numpy, the arithmetic the reference (lizaibeim/mmla-audio) runs on the
per-clip path "WAV -> features -> Keras net -> class".  It is the *checker*: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.  The product
(``mmla_audio_amd``) never imports, links or falls back to anything in here.

Modules
-------
od_fe   librosa 0.8.x restatement of the OverlapDetection front-end
        (reference: OverlapDetection/scripts/overlap_features_generator.py:65-151).
si_fe   python_speech_features 0.6 restatement of the SpeakerIdentification front-end
        (reference: SpeakerIdentification/scripts/speaker_identification.py:141-151,372-398).
nets    numpy restatement of the two Keras graphs in inference mode
        (reference: OverlapDetection/scripts/overlap_detector_temp.py:253-303,
        SpeakerIdentification/scripts/speaker_identification.py:168-218,401-410).
synth   deterministic synthetic 16 kHz int16 clips.

Pinning
-------
The reference has no tests and no golden vectors.  The reference's *own*
numpy glue (pad/trunc, normalize_matrix, image assembly, delta, the 'silent' gate, the
matplotlib PNG quantisation) is pinned by running the reference source itself in this container
with the absent third-party modules replaced by these restatements
(``tests/golden/make_golden.py``).  The third-party arithmetic (librosa, python_speech_features,
TF/Keras) is not installed anywhere in this image, so that part is a restatement of the
published algorithms and is *parity unpinned* by any reference-held fixture.
"""
