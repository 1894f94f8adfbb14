"""WAV I/O (io/wav.{h,cc} restated natively in libcrlot_dsp.so; host only).

Mirrors the reference's tests/wav_io_test.cc cases (oboe.wav info and data,
invalid files, write -> read round trips at 16/24/32 bit, mono, empty, sample
rates) and pins the conversions exactly: reading against Python's stdlib
`wave` decoder (an independent RIFF parser), writing against the published
dr_wav / wav.cc formulas.  dr_wav itself (third_party/dr_libs, an empty
submodule) is absent, so the dr_wav-side formulas are restated, not run.
tests/golden/oboe.wav is the reference's own assets/oboe.wav (data fixture).
"""
import os
import struct
import wave

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
OBOE = os.path.join(GOLD, "oboe.wav")


def test_oboe_info_and_data(pkg):
    """wav_io_test.cc:34-90 (+ SURVEY 8d config 1: 2 ch, 44.1 kHz, s16, 285315 frames)."""
    r = pkg.WavReader()
    assert r.open(OBOE) and r.is_open()
    assert (r.get_channels(), r.get_sample_rate(), r.get_bits_per_sample()) == (2, 44100, 16)
    assert r.get_total_frames() == 285315
    data = r.read_all()
    assert data.size == 285315 * 2
    with wave.open(OBOE, "rb") as w:
        raw = np.frombuffer(w.readframes(w.getnframes()), "<i2")
    assert np.array_equal(data, raw.astype(np.float32) / np.float32(32768))  # drwav_s16_to_f32
    r.close()
    assert not r.is_open()


def test_chunked_reads_equal_read_all(pkg):
    r = pkg.WavReader()
    assert r.open(OBOE)
    parts = []
    while True:
        p = r.read(10_000)
        if p.size == 0:
            break
        parts.append(p)
    r.close()
    r.open(OBOE)
    assert np.array_equal(np.concatenate(parts), r.read_all())


def test_mono_mixdown_matches_main_cc(pkg):
    """main/main.cc:155-160: (L + R) summed in float, / channels."""
    x, sr = pkg.load_wav_mono(OBOE)
    with wave.open(OBOE, "rb") as w:
        raw = np.frombuffer(w.readframes(w.getnframes()), "<i2").reshape(-1, 2)
    f = raw.astype(np.float32) / np.float32(32768)
    ref = ((np.float32(0) + f[:, 0]).astype(np.float32) + f[:, 1]).astype(np.float32) / np.float32(2)
    assert sr == 44100 and np.array_equal(x, ref.astype(np.float32))


def test_open_invalid(pkg, tmp_path):
    r = pkg.WavReader()
    assert not r.open("nonexistent.wav") and not r.is_open()
    bad = tmp_path / "junk.wav"
    bad.write_bytes(b"not a wav file at all")
    assert not r.open(bad)
    # guards of WavReader::open: 8-bit and 3-channel files are refused
    for ch, width in ((1, 1), (3, 2)):
        p = tmp_path / f"g_{ch}_{width}.wav"
        with wave.open(str(p), "wb") as w:
            w.setnchannels(ch)
            w.setsampwidth(width)
            w.setframerate(8000)
            w.writeframes(b"\x00" * (ch * width * 10))
        assert not r.open(p), (ch, width)
        assert r.last_error


def _f32_to_s16(x):
    c = np.clip(x.astype(np.float32), np.float32(-1), np.float32(1)) + np.float32(1)
    return ((c * np.float32(32767.5)).astype(np.int32) - 32768).astype(np.int16)


def _rand(frames, ch, seed=42):
    rng = np.random.default_rng(seed)
    return ((rng.random(frames * ch, dtype=np.float32) - np.float32(0.5)) * np.float32(0.8))


def _roundtrip(pkg, path, data, ch, rate, bits, float_format=False):
    w = pkg.WavWriter()
    assert w.open(path, ch, rate, bits, float_format) and w.is_open()
    assert w.write(data) == data.size // ch
    w.close()
    assert not w.is_open()
    r = pkg.WavReader()
    assert r.open(path)
    assert (r.get_channels(), r.get_sample_rate(), r.get_bits_per_sample(),
            r.get_total_frames()) == (ch, rate, bits, data.size // ch)
    out = r.read_all()
    r.close()
    return out


def test_write_read_16bit(pkg, tmp_path):
    """wav_io_test.cc:94-144 and :214-297 (16-bit, stereo, 44.1/48 kHz)."""
    t = np.arange(44100, dtype=np.float32)
    s = (0.5 * np.sin(2 * np.float32(np.pi) * 440 * t / 44100)).astype(np.float32)
    data = np.stack([s, s], 1).reshape(-1)
    out = _roundtrip(pkg, tmp_path / "a.wav", data, 2, 44100, 16)
    assert np.max(np.abs(out - data)) < 0.01
    exp = _f32_to_s16(data).astype(np.float32) / np.float32(32768)
    assert np.array_equal(out, exp)  # drwav_f32_to_s16 then s16 * 2^-15
    # the header is a valid RIFF/WAVE for an independent decoder
    with wave.open(str(tmp_path / "a.wav"), "rb") as w:
        assert (w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()) == (2, 2, 44100, 44100)
        assert np.array_equal(np.frombuffer(w.readframes(44100), "<i2"), _f32_to_s16(data))
    for rate in (44100, 48000):
        d = _rand(1000, 2)
        o = _roundtrip(pkg, tmp_path / f"r{rate}.wav", d, 2, rate, 16)
        err = o.astype(np.float64) - d
        assert np.max(np.abs(err)) < 0.001
        assert 10 * np.log10(np.sum(d.astype(np.float64) ** 2) / np.sum(err ** 2)) > 60.0


def test_write_read_mono_and_empty(pkg, tmp_path):
    """wav_io_test.cc:146-198."""
    t = np.arange(22050 // 2, dtype=np.float32)
    d = (0.3 * np.sin(2 * np.float32(np.pi) * 880 * t / 22050)).astype(np.float32)
    _roundtrip(pkg, tmp_path / "m.wav", d, 1, 22050, 16)
    out = _roundtrip(pkg, tmp_path / "e.wav", np.zeros(0, np.float32), 1, 44100, 16)
    assert out.size == 0


def test_write_read_24_and_32bit(pkg, tmp_path):
    """wav_io_test.cc BitDepth_24Bit / 32Bit round trips, plus the exact codes."""
    d = _rand(1000, 2, seed=7)
    d[:4] = [1.5, -1.5, 1.0, -1.0]  # clamping
    o24 = _roundtrip(pkg, tmp_path / "b24.wav", d, 2, 44100, 24)
    codes = np.rint(np.clip(d, -1, 1).astype(np.float32) * np.float32(8388607)).astype(np.int64)
    assert np.array_equal(o24, (codes.astype(np.float64) / 8388608).astype(np.float32))
    assert np.max(np.abs(o24[4:] - d[4:])) < 1e-4
    with wave.open(str(tmp_path / "b24.wav"), "rb") as w:
        raw = np.frombuffer(w.readframes(w.getnframes()), np.uint8).reshape(-1, 3).astype(np.int32)
        v = (raw[:, 0] | (raw[:, 1] << 8) | (raw[:, 2] << 16))
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        assert np.array_equal(v, codes)
    o32 = _roundtrip(pkg, tmp_path / "b32.wav", d, 2, 44100, 32)
    assert np.max(np.abs(o32[4:] - d[4:])) < 1e-5
    assert o32[0] == np.float32(2147483647 / 2147483648) and o32[1] == -1.0
    of = _roundtrip(pkg, tmp_path / "f32.wav", d, 2, 44100, 32, float_format=True)
    assert np.array_equal(of, d)  # IEEE float: bit exact


def test_writer_guards(pkg, tmp_path):
    w = pkg.WavWriter()
    assert not w.open(tmp_path / "x.wav", 3, 44100, 16)
    assert not w.open(tmp_path / "x.wav", 1, 44100, 8)
    assert not w.open(tmp_path / "x.wav", 0, 44100, 16)


def test_extensible_and_extra_chunks(pkg, tmp_path):
    """WAVE_FORMAT_EXTENSIBLE (fmt size 40, SubFormat = PCM) and a LIST chunk
    before the data, as written by many tools: parsed like dr_wav does."""
    pcm = (np.arange(20, dtype=np.int16) * 100 - 1000)
    fmt = struct.pack("<HHIIHH", 0xFFFE, 2, 16000, 16000 * 4, 4, 16)
    fmt += struct.pack("<HHI", 22, 16, 3) + struct.pack("<H", 1) + bytes(14)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt
    body += b"LIST" + struct.pack("<I", 5) + b"INFOx" + b"\x00"  # odd size + pad byte
    body += b"data" + struct.pack("<I", pcm.nbytes) + pcm.tobytes()
    p = tmp_path / "ext.wav"
    p.write_bytes(b"RIFF" + struct.pack("<I", len(body)) + body)
    r = pkg.WavReader()
    assert r.open(p)
    assert (r.get_channels(), r.get_sample_rate(), r.get_total_frames()) == (2, 16000, 10)
    assert np.array_equal(r.read_all(), pcm.astype(np.float32) / 32768)
