"""WebRTC voice activity detector (py-webrtcvad 2.0.10 / WebRTC common_audio/vad) restated in pure
Python integer arithmetic -- TEST INFRASTRUCTURE ONLY.

The reference calls ``webrtcvad.Vad(3).is_speech(frame_bytes, 16000)`` on 30 ms frames
(``OverlapDetection/scripts/record_on_pc.py:33,256``; ``overlap_detection_post_processing.py:17,140``;
SpeakerIdentification ``record_on_pc.py:31,234``, ``speaker_identification_post_processing.py:26,
180,236``).  webrtcvad is a C extension that is absent from this image (and not in
/root/reference), so this is a restatement of the library's published fixed-point algorithm
(vad_core.c GmmProbability / CalcVad16khz, vad_filterbank.c CalculateFeatures, vad_gmm.c
GaussianProbability, vad_sp.c Downsampling / FindMinimum, signal_processing Energy / Norm / Div)
from the WebRTC sources as published: **parity unpinned** (no reference vector exists).  It fixes
the semantics the HIP kernel (mmla_audio_amd/csrc/vad.hip) reproduces bit for bit.

C integer semantics are emulated: int16_t stores wrap (``_s16``), int32 products wrap (``_s32``),
``>>`` is arithmetic, divisions truncate toward zero (``_div``).  A Vad keeps its state across
calls exactly like the module-level ``vad`` object of the reference scripts.
"""
import numpy as np

K_NUM_CHANNELS, K_NUM_GAUSSIANS = 6, 2
K_TABLE = K_NUM_CHANNELS * K_NUM_GAUSSIANS
K_MIN_ENERGY = 10

SPECTRUM_WEIGHT = (6, 8, 10, 12, 14, 16)
NOISE_UPDATE, SPEECH_UPDATE, BACK_ETA = 655, 6554, 154
MINIMUM_DIFFERENCE = (544, 544, 576, 576, 576, 576)
MAXIMUM_SPEECH = (11392, 11392, 11520, 11520, 11520, 11520)
MINIMUM_MEAN = (640, 768)
MAXIMUM_NOISE = (9216, 9088, 8960, 8832, 8704, 8576)
NOISE_WEIGHTS = (34, 62, 72, 66, 53, 25, 94, 66, 56, 62, 75, 103)
SPEECH_WEIGHTS = (48, 82, 45, 87, 50, 47, 80, 46, 83, 41, 78, 81)
NOISE_MEANS = (6738, 4892, 7065, 6715, 6771, 3369, 7646, 3863, 7820, 7266, 5020, 4362)
SPEECH_MEANS = (8306, 10085, 10078, 11823, 11843, 6309, 9473, 9571, 10879, 7581, 8180, 7483)
NOISE_STDS = (378, 1064, 493, 582, 688, 593, 474, 697, 475, 688, 421, 455)
SPEECH_STDS = (555, 505, 567, 524, 585, 1231, 509, 828, 492, 1540, 1079, 850)
MAX_SPEECH_FRAMES, MIN_STD = 6, 384
# per mode: over_hang_max_1, over_hang_max_2, individual, total; entries for 10 / 20 / 30 ms
MODES = {
    0: ((8, 4, 3), (14, 7, 5), (24, 21, 24), (57, 48, 57)),
    1: ((8, 4, 3), (14, 7, 5), (37, 32, 37), (100, 80, 100)),
    2: ((6, 3, 2), (9, 5, 3), (82, 78, 82), (285, 260, 285)),
    3: ((6, 3, 2), (9, 5, 3), (94, 94, 94), (1100, 1050, 1100)),
}
COMP_VAR, LOG2_EXP = 22005, 5909
SMOOTHING_DOWN, SMOOTHING_UP = 6553, 32439
ALLPASS_Q13 = (5243, 1392)          # 16 -> 8 kHz downsampler
ALLPASS_Q15 = (20972, 5571)         # splitting filter, upper / lower branch
HP_ZERO = (6631, -13262, 6631)
HP_POLE = (16384, -7756, 5620)
OFFSET_VECTOR = (368, 368, 272, 176, 176, 176)
LOG_CONST, LOG_ENERGY_INT = 24660, 14336


def _s16(x):
    x &= 0xFFFF
    return x - 0x10000 if x & 0x8000 else x


def _s32(x):
    x &= 0xFFFFFFFF
    return x - 0x100000000 if x & 0x80000000 else x


def _div(num, den):
    """WebRtcSpl_DivW32W16: C division (truncation toward zero); 0x7FFFFFFF for den == 0"""
    if den == 0:
        return 0x7FFFFFFF
    q = abs(num) // abs(den)
    return q if (num >= 0) == (den > 0) else -q


def _norm_w32(a):
    """WebRtcSpl_NormW32: left shifts that normalise a signed 32-bit value (0 -> 0)"""
    a = _s32(a)
    if a == 0:
        return 0
    if a < 0:
        a = ~a
    return 32 - a.bit_length() - 1 if a else 31


def _norm_u32(a):
    return 0 if a == 0 else 32 - (a & 0xFFFFFFFF).bit_length()


def _size_in_bits(n):
    return n.bit_length()


def _energy(x):
    """WebRtcSpl_Energy with GetScalingSquare: -> (energy, scaling)"""
    smax = -1
    for v in x:
        sabs = _s16(-v) if v <= 0 else v
        smax = max(smax, sabs)
    nbits = _size_in_bits(len(x))
    t = _norm_w32(smax * smax)
    scaling = 0 if smax == 0 else (0 if t > nbits else nbits - t)
    en = 0
    for v in x:
        en = _s32(en + ((v * v) >> scaling))
    return en, scaling


class Vad:
    """webrtcvad.Vad(mode): WebRtcVad_Create + InitCore + set_mode_core"""

    def __init__(self, mode=3):
        if mode not in MODES:
            raise ValueError(mode)
        self.mode = mode
        self.oh1, self.oh2, self.individual, self.total = MODES[mode]
        self.frame_counter = 0
        self.over_hang = 0
        self.num_of_speech = 0
        self.ds_state = [0, 0]
        self.noise_means = list(NOISE_MEANS)
        self.speech_means = list(SPEECH_MEANS)
        self.noise_stds = list(NOISE_STDS)
        self.speech_stds = list(SPEECH_STDS)
        self.low_value = [10000] * (16 * K_NUM_CHANNELS)
        self.index = [0] * (16 * K_NUM_CHANNELS)
        self.upper_state = [0] * 5
        self.lower_state = [0] * 5
        self.hp_state = [0] * 4
        self.mean_value = [1600] * K_NUM_CHANNELS

    # ---- signal processing (vad_sp.c, vad_filterbank.c) -------------------------------------------
    def _downsample(self, x):
        t1, t2 = self.ds_state
        out = []
        for n in range(len(x) // 2):
            a = _s16((t1 >> 1) + ((ALLPASS_Q13[0] * x[2 * n]) >> 14))
            t1 = _s32(x[2 * n] - ((ALLPASS_Q13[0] * a) >> 12))
            b = _s16((t2 >> 1) + ((ALLPASS_Q13[1] * x[2 * n + 1]) >> 14))
            t2 = _s32(x[2 * n + 1] - ((ALLPASS_Q13[1] * b) >> 12))
            out.append(_s16(a + b))
        self.ds_state = [t1, t2]
        return out

    @staticmethod
    def _allpass(x, start, n, coef, state):
        s32 = _s32(state * 65536)
        out = []
        for i in range(n):
            v = x[start + 2 * i]
            t32 = _s32(s32 + coef * v)
            t16 = _s16(t32 >> 16)
            out.append(t16)
            s32 = _s32((v * 16384 - coef * t16) * 2)
        return out, _s16(s32 >> 16)

    def _split(self, x, band):
        half = len(x) // 2
        hp, self.upper_state[band] = self._allpass(x, 0, half, ALLPASS_Q15[0], self.upper_state[band])
        lp, self.lower_state[band] = self._allpass(x, 1, half, ALLPASS_Q15[1], self.lower_state[band])
        return [_s16(h - l) for h, l in zip(hp, lp)], [_s16(l + h) for h, l in zip(hp, lp)]

    def _highpass(self, x):
        st = self.hp_state
        out = []
        for v in x:
            t = HP_ZERO[0] * v + HP_ZERO[1] * st[0] + HP_ZERO[2] * st[1]
            st[1], st[0] = st[0], v
            t = _s32(t - HP_POLE[1] * st[2] - HP_POLE[2] * st[3])
            st[3] = st[2]
            st[2] = _s16(t >> 14)
            out.append(st[2])
        return out

    @staticmethod
    def _log_energy(x, offset, total):
        energy, tot_rshifts = _energy(x)
        energy &= 0xFFFFFFFF
        if energy == 0:
            return offset, total
        nr = 17 - _norm_u32(energy)
        log2_energy = LOG_ENERGY_INT
        tot_rshifts += nr
        energy = (energy << -nr) & 0xFFFFFFFF if nr < 0 else energy >> nr
        log2_energy = _s16(log2_energy + ((energy & 0x3FFF) >> 4))
        le = _s16(((LOG_CONST * log2_energy) >> 19) + ((tot_rshifts * LOG_CONST) >> 9))
        if le < 0:
            le = 0
        le = _s16(le + offset)
        if total <= K_MIN_ENERGY:
            if tot_rshifts >= 0:
                total = _s16(total + K_MIN_ENERGY + 1)
            else:
                total = _s16(total + _s16(energy >> -tot_rshifts))
        return le, total

    def _features(self, x):
        feats = [0] * K_NUM_CHANNELS
        total = 0
        hp120, lp120 = self._split(x, 0)              # 2000-4000 / 0-2000 Hz
        hp60, lp60 = self._split(hp120, 1)            # 3000-4000 / 2000-3000
        feats[5], total = self._log_energy(hp60, OFFSET_VECTOR[5], total)
        feats[4], total = self._log_energy(lp60, OFFSET_VECTOR[4], total)
        hp60, lp60 = self._split(lp120, 2)            # 1000-2000 / 0-1000
        feats[3], total = self._log_energy(hp60, OFFSET_VECTOR[3], total)
        hp120, lp120 = self._split(lp60, 3)           # 500-1000 / 0-500
        feats[2], total = self._log_energy(hp120, OFFSET_VECTOR[2], total)
        hp60, lp60 = self._split(lp120, 4)            # 250-500 / 0-250
        feats[1], total = self._log_energy(hp60, OFFSET_VECTOR[1], total)
        feats[0], total = self._log_energy(self._highpass(lp60), OFFSET_VECTOR[0], total)
        return feats, total

    # ---- the GMM (vad_gmm.c, vad_core.c, vad_sp.c) -------------------------------------------------
    @staticmethod
    def _gauss(x, mean, std):
        inv_std = _s16(_div(131072 + (std >> 1), std))
        t16 = inv_std >> 2
        inv_std2 = _s16((t16 * t16) >> 2)
        t16 = _s16(_s16(x << 3) - mean)
        delta = _s16((inv_std2 * t16) >> 10)
        t32 = (delta * t16) >> 9
        exp_value = 0
        if t32 < COMP_VAR:
            t16 = _s16((LOG2_EXP * t32) >> 12)
            t16 = _s16(-t16)
            exp_value = 0x0400 | (t16 & 0x03FF)
            t16 = _s16(t16 ^ 0xFFFF)
            t16 >>= 10
            t16 += 1
            exp_value >>= t16
        return _s32(inv_std * exp_value), delta

    def _find_minimum(self, value, ch):
        off = ch * 16
        age = self.index
        sv = self.low_value
        i = 0
        while i < 16:
            if age[off + i] != 100:
                age[off + i] += 1
            else:
                for j in range(i, 15):
                    sv[off + j] = sv[off + j + 1]
                    age[off + j] = age[off + j + 1]
                age[off + 15] = 101
                sv[off + 15] = 10000
            i += 1
        pos = -1
        for p in range(16):
            if value < sv[off + p]:
                pos = p
                break
        if pos > -1:
            for i in range(15, pos, -1):
                sv[off + i] = sv[off + i - 1]
                age[off + i] = age[off + i - 1]
            sv[off + pos] = value
            age[off + pos] = 1
        median = 1600
        if self.frame_counter > 2:
            median = sv[off + 2]
        elif self.frame_counter > 0:
            median = sv[off + 0]
        alpha = 0
        if self.frame_counter > 0:
            alpha = SMOOTHING_DOWN if median < self.mean_value[ch] else SMOOTHING_UP
        t32 = (alpha + 1) * self.mean_value[ch] + (32767 - alpha) * median + 16384
        self.mean_value[ch] = _s16(t32 >> 15)
        return self.mean_value[ch]

    def _wavg(self, data, ch, offset, weights):
        s = 0
        for k in range(K_NUM_GAUSSIANS):
            g = ch + k * K_NUM_CHANNELS
            data[g] = _s16(data[g] + offset)
            s += data[g] * weights[g]
        return s

    def _gmm(self, feats, total_power, fi):
        oh1, oh2, individual, total_test = self.oh1[fi], self.oh2[fi], self.individual[fi], self.total[fi]
        vadflag = 0
        if total_power > K_MIN_ENERGY:
            delta_n, delta_s = [0] * K_TABLE, [0] * K_TABLE
            ngpr, sgpr = [0] * K_TABLE, [0] * K_TABLE
            sum_llr = 0
            for ch in range(K_NUM_CHANNELS):
                h0t = h1t = 0
                npb, spb = [0, 0], [0, 0]
                for k in range(K_NUM_GAUSSIANS):
                    g = ch + k * K_NUM_CHANNELS
                    p, delta_n[g] = self._gauss(feats[ch], self.noise_means[g], self.noise_stds[g])
                    npb[k] = _s32(NOISE_WEIGHTS[g] * p)
                    h0t = _s32(h0t + npb[k])
                    p, delta_s[g] = self._gauss(feats[ch], self.speech_means[g], self.speech_stds[g])
                    spb[k] = _s32(SPEECH_WEIGHTS[g] * p)
                    h1t = _s32(h1t + spb[k])
                sh0 = 31 if h0t == 0 else _norm_w32(h0t)
                sh1 = 31 if h1t == 0 else _norm_w32(h1t)
                llr = _s16(sh0 - sh1)
                sum_llr += llr * SPECTRUM_WEIGHT[ch]
                if llr * 4 > individual:
                    vadflag = 1
                h0 = _s16(h0t >> 12)
                if h0 > 0:
                    t = _s32((npb[0] & 0xFFFFF000) << 2)
                    ngpr[ch] = _s16(_div(t, h0))
                    ngpr[ch + K_NUM_CHANNELS] = _s16(16384 - ngpr[ch])
                else:
                    ngpr[ch] = 16384
                h1 = _s16(h1t >> 12)
                if h1 > 0:
                    t = _s32((spb[0] & 0xFFFFF000) << 2)
                    sgpr[ch] = _s16(_div(t, h1))
                    sgpr[ch + K_NUM_CHANNELS] = _s16(16384 - sgpr[ch])
            vadflag |= int(sum_llr >= total_test)

            maxspe = 12800
            for ch in range(K_NUM_CHANNELS):
                fmin = self._find_minimum(feats[ch], ch)
                ngm = self._wavg(self.noise_means, ch, 0, NOISE_WEIGHTS)
                t1 = _s16(ngm >> 6)
                for k in range(K_NUM_GAUSSIANS):
                    g = ch + k * K_NUM_CHANNELS
                    nmk, smk = self.noise_means[g], self.speech_means[g]
                    nsk, ssk = self.noise_stds[g], self.speech_stds[g]
                    nmk2 = nmk
                    if not vadflag:
                        delt = _s16((ngpr[g] * delta_n[g]) >> 11)
                        nmk2 = _s16(nmk + _s16((delt * NOISE_UPDATE) >> 22))
                    ndelt = _s16((fmin << 4) - t1)
                    nmk3 = _s16(nmk2 + _s16((ndelt * BACK_ETA) >> 9))
                    lo = _s16((k + 5) << 7)
                    if nmk3 < lo:
                        nmk3 = lo
                    hi = _s16((72 + k - ch) << 7)
                    if nmk3 > hi:
                        nmk3 = hi
                    self.noise_means[g] = nmk3
                    if vadflag:
                        delt = _s16((sgpr[g] * delta_s[g]) >> 11)
                        t16 = _s16((delt * SPEECH_UPDATE) >> 21)
                        smk2 = _s16(smk + ((t16 + 1) >> 1))
                        maxmu = maxspe + 640
                        if smk2 < MINIMUM_MEAN[k]:
                            smk2 = MINIMUM_MEAN[k]
                        if smk2 > maxmu:
                            smk2 = maxmu
                        self.speech_means[g] = smk2
                        t16 = (smk + 4) >> 3
                        t16 = _s16(feats[ch] - t16)
                        t1_32 = (delta_s[g] * t16) >> 3
                        t2_32 = t1_32 - 4096
                        t16 = sgpr[g] >> 2
                        t1_32 = _s32(t16 * t2_32)
                        t2_32 = t1_32 >> 4
                        if t2_32 > 0:
                            t16 = _s16(_div(t2_32, _s16(ssk * 10)))
                        else:
                            t16 = _s16(-_s16(_div(-t2_32, _s16(ssk * 10))))
                        t16 = _s16(t16 + 128)
                        ssk = _s16(ssk + (t16 >> 8))
                        if ssk < MIN_STD:
                            ssk = MIN_STD
                        self.speech_stds[g] = ssk
                    else:
                        t16 = _s16(feats[ch] - (nmk >> 3))
                        t1_32 = (delta_n[g] * t16) >> 3
                        t1_32 -= 4096
                        t16 = (ngpr[g] + 2) >> 2
                        t2_32 = _s32(t16 * t1_32)
                        t1_32 = t2_32 >> 14
                        if t1_32 > 0:
                            t16 = _s16(_div(t1_32, nsk))
                        else:
                            t16 = _s16(-_s16(_div(-t1_32, nsk)))
                        t16 = _s16(t16 + 32)
                        nsk = _s16(nsk + (t16 >> 6))
                        if nsk < MIN_STD:
                            nsk = MIN_STD
                        self.noise_stds[g] = nsk
                ngm = self._wavg(self.noise_means, ch, 0, NOISE_WEIGHTS)
                sgm = self._wavg(self.speech_means, ch, 0, SPEECH_WEIGHTS)
                diff = _s16(_s16(sgm >> 9) - _s16(ngm >> 9))
                if diff < MINIMUM_DIFFERENCE[ch]:
                    t16 = MINIMUM_DIFFERENCE[ch] - diff
                    a = _s16((13 * t16) >> 2)
                    b = _s16((3 * t16) >> 2)
                    sgm = self._wavg(self.speech_means, ch, a, SPEECH_WEIGHTS)
                    ngm = self._wavg(self.noise_means, ch, -b, NOISE_WEIGHTS)
                maxspe = MAXIMUM_SPEECH[ch]
                t2 = _s16(sgm >> 7)
                if t2 > maxspe:
                    t2 -= maxspe
                    for k in range(K_NUM_GAUSSIANS):
                        g = ch + k * K_NUM_CHANNELS
                        self.speech_means[g] = _s16(self.speech_means[g] - t2)
                t2 = _s16(ngm >> 7)
                if t2 > MAXIMUM_NOISE[ch]:
                    t2 -= MAXIMUM_NOISE[ch]
                    for k in range(K_NUM_GAUSSIANS):
                        g = ch + k * K_NUM_CHANNELS
                        self.noise_means[g] = _s16(self.noise_means[g] - t2)
            self.frame_counter += 1
        if not vadflag:
            if self.over_hang > 0:
                vadflag = 2 + self.over_hang
                self.over_hang -= 1
            self.num_of_speech = 0
        else:
            self.num_of_speech += 1
            if self.num_of_speech > MAX_SPEECH_FRAMES:
                self.num_of_speech = MAX_SPEECH_FRAMES
                self.over_hang = oh2
            else:
                self.over_hang = oh1
        return vadflag

    def is_speech(self, frame, sample_rate=16000):
        """one 10/20/30 ms frame of int16 PCM (bytes or array) at 16 kHz -> bool"""
        if sample_rate != 16000:
            raise ValueError('this restatement covers the 16 kHz path the reference uses')
        x = np.frombuffer(frame, dtype='<i2') if isinstance(frame, (bytes, bytearray)) else np.asarray(frame)
        if len(x) not in (160, 320, 480):
            raise ValueError('frame must be 10, 20 or 30 ms')
        x8 = self._downsample([int(v) for v in x])
        feats, total = self._features(x8)
        return self._gmm(feats, total, {80: 0, 160: 1, 240: 2}[len(x8)]) > 0
