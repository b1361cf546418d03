/* Host-side input pipeline of the north-star path: the arithmetic of
 * src/data/ravdess.py's load_audio_wav / load_video_frames that runs on the CPU before a clip reaches the GPU,
 * as plain C entry points (libmer_io.so, g++, no GPU, no torch types).  The device side -- pad / crop of the
 * waveforms, face-box crop + resize + ImageNet normalisation of the frames -- is in mer.h (csrc/clips.hip).
 * Every function returns 0 on success or a negative MER_IO_* code. */
#ifndef MER_IO_H
#define MER_IO_H

#ifdef __cplusplus
extern "C" {
#endif

#define MER_IO_OK 0
#define MER_IO_EOPEN -1     /* cannot open / read the file */
#define MER_IO_EFORMAT -2   /* not a RIFF/WAVE file, or an unsupported sample format */
#define MER_IO_EARG -3      /* bad argument (NULL pointer, capacity too small, rate <= 0) */

/* WAV header: sample rate, channel count, frames per channel, sample format (1 = integer PCM, 3 = IEEE float;
 * WAVE_FORMAT_EXTENSIBLE is resolved to its sub-format) and bits per sample.  Replaces the header half of
 * librosa.load -> soundfile.read (ravdess.py:505). */
int mer_wav_info(const char* path, int* sample_rate, int* channels, long long* frames, int* format, int* bits);

/* Decode a WAV file to mono float32: samples scaled like soundfile's float reads (integer PCM / 2^(bits-1),
 * 8-bit unsigned centred at 128, float data as stored), channels averaged (librosa.to_mono: mean over the
 * channel axis).  out needs `frames` floats (mer_wav_info); *n_out = frames written.  (ravdess.py:505) */
int mer_wav_read_mono(const char* path, float* out, long long capacity, long long* n_out);

/* Polyphase rational resampling sr_in -> sr_out of a mono float32 signal, scipy.signal.resample_poly's
 * algorithm (Kaiser(beta 5) windowed-sinc FIR of 20*max(up,down)+1 taps, cutoff 1/max(up,down), zero padding),
 * n_out = ceil(n_in * sr_out / sr_in).  Stands in for librosa.load's resampler (soxr_hq, absent from this
 * image: parity unpinned; pinned against scipy here).  out needs mer_resample_len(...) floats. */
long long mer_resample_len(long long n_in, int sr_in, int sr_out);
int mer_resample(const float* in, long long n_in, int sr_in, int sr_out, float* out, long long capacity,
                 long long* n_out);

/* _uniform_indices (ravdess.py:272-277): `num` frame indices spread over `total` frames --
 * round(linspace(0, total-1, num)) with round-half-to-even when total >= num, else 0..total-1 then the last
 * index repeated; total <= 0 gives zeros. */
int mer_uniform_indices(int total, int num, int* out);

/* crop_with_padding's box (face_crop.py:151-190): the (x1, y1, x2, y2) bbox padded by int(bbox_w * pad_ratio) /
 * int(bbox_h * pad_ratio) on each side and clipped to the w x h frame -> out[4] = (x1, y1, x2, y2). */
int mer_face_crop_box(int h, int w, int x1, int y1, int x2, int y2, float pad_ratio, int* out);

/* Bar-noise augmentation of load_audio_wav (ravdess.py:543-566): wav[i] = clamp(wav[i] + s * noise[start + i],
 * -1, 1) with s = sqrt((P_sig / 10^(snr_db/10)) / P_noise) (s = 1 when P_noise <= 1e-8), P = mean of squares
 * (noise tiled when shorter than n).  In place. */
int mer_mix_noise(float* wav, long long n, const float* noise, long long n_noise, long long start, float snr_db);

#ifdef __cplusplus
}
#endif
#endif
