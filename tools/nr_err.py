import sys, numpy as np
sys.path.insert(0, '.')
from oracle import noisereduce as onr, synth
from mmla_audio_amd import noisereduce as nr
rng = np.random.default_rng(5)
noise = (0.01 * rng.standard_normal(48000)).astype(np.float32)
for seed in range(6):
    y = (synth.clip(300 + seed, 40000).astype(np.float32) / 32768.0 + 0.01 * rng.standard_normal(40000)).astype(np.float32)
    g = nr.reduce_noise(y=y, sr=16000, y_noise=noise, stationary=True)
    w = onr.reduce_noise(y, 16000, noise)
    print(seed, 'max abs err', float(np.abs(g - w).max()), 'peak', float(np.abs(w).max()), 'rms in/out', float(np.sqrt(np.mean(y**2))), float(np.sqrt(np.mean(w**2))))
