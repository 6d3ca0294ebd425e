"""The output leg after the decode: what the reference does with every song
once the VAE is done, on MI355X.

Reference, per song (``acestep/inference.py:673-716``, ``acestep/audio_utils.py:24-210``,
``generate_music_payload.py:41``):
  1. ``pred_wavs[i].cpu()`` — the fp32 audio [2, 1920·T] to the host (92 MB at 240 s);
  2. ``normalize_audio(audio, normalization_db)`` on the host (clone, max |x|, multiply);
  3. ``AudioSaver.save_audio`` → ``audio.cpu().float().contiguous()`` → soundfile, which takes
     [samples, channels] frames and converts each float sample to PCM16 (the FLAC / WAV
     default subtype) before encoding and writing the file.

Here: steps 2 and the sample conversion of 3 run on the GPU in the postprocess pass pair
(``acehip_wav_postprocess_pcm16``: peak guard + normalize + interleaved PCM16 frames), so the
device→host copy carries 46 MB instead of 92 MB per 240 s song, into pinned memory on a side
stream, and a host thread writes the file — while the GPU already runs the next song.
``soundfile`` / ``torchaudio`` (the FLAC encoder) are not installed in this image, so files are
written as PCM16 WAV with the stdlib ``wave`` module; a FLAC encoder would take the same
interleaved frames.
"""
from __future__ import annotations

import os
import queue
import threading
import wave
from typing import List, Optional, Sequence

import torch

from ._ffi import check, lib, ptr, stream_ptr


def target_amp(normalization_db: Optional[float]) -> float:
    """fp32(10^(db/20)) as torch evaluates ``target_amp / peak`` (audio_utils.py:54-57); None = no
    normalisation (the decode guard only)."""
    if normalization_db is None:
        return 0.0
    if normalization_db > 0.0:
        raise ValueError("normalization_db must be <= 0 (inference.py:674)")
    return float(torch.tensor(10 ** (normalization_db / 20.0), dtype=torch.float32))


def postprocess_pcm16_(wav: torch.Tensor, normalization_db: Optional[float] = -1.0,
                       pcm: Optional[torch.Tensor] = None) -> torch.Tensor:
    """In place on ``wav`` (fp32 [B, C, N] on the device): the decode guard + normalize_audio, as
    ``OobleckBackend.postprocess_``; returns the PCM16 frames [B, N, C] (int16, device) of the
    result, rint(clamp(x, −1, 1)·32767)."""
    assert wav.is_cuda and wav.dtype == torch.float32 and wav.is_contiguous() and wav.dim() == 3
    B, C, N = wav.shape
    if pcm is None:
        pcm = torch.empty(B, N, C, device=wav.device, dtype=torch.int16)
    assert pcm.shape == (B, N, C) and pcm.dtype == torch.int16 and pcm.is_contiguous()
    peak = torch.empty(B, device=wav.device, dtype=torch.float32)
    check(lib().acehip_wav_postprocess_pcm16(ptr(wav), B, C, N, ptr(peak), 1, target_amp(normalization_db),
                                             ptr(pcm), stream_ptr()), "wav_postprocess_pcm16")
    return pcm


def write_wav_pcm16(path: str, frames, sample_rate: int = 48000, channels: int = 2) -> str:
    """Write interleaved PCM16 frames (host int16 tensor / array [N, C]) as a WAV file."""
    buf = frames.numpy() if isinstance(frames, torch.Tensor) else frames
    with wave.open(path, "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(2)
        w.setframerate(sample_rate)
        w.writeframes(memoryview(buf).cast("B"))
    return path


class AudioWriter:
    """Asynchronous output leg: ``submit(wav, paths)`` right after a song's decode; the guard +
    normalize + PCM16 pack runs on the caller's stream, the device→host copy of the frames on a
    side stream into a pinned host slot, and a writer thread saves the WAV once the copy is done.
    The caller's stream goes straight on to the next song; ``flush()`` waits for every file.

    Slots are reused round-robin (``slots`` songs in flight); ``submit`` blocks only when all of
    them still wait for their file write."""

    def __init__(self, device: torch.device, max_frames: int, channels: int = 2, slots: int = 2,
                 sample_rate: int = 48000, normalization_db: Optional[float] = -1.0):
        self.device = device
        self.C, self.sr, self.db = channels, sample_rate, normalization_db
        self.copy_stream = torch.cuda.Stream(device=device)
        self.host = [torch.empty(max_frames * channels, dtype=torch.int16, pin_memory=True) for _ in range(slots)]
        self.pcm = [torch.empty(max_frames * channels, dtype=torch.int16, device=device) for _ in range(slots)]
        self.free: "queue.Queue[int]" = queue.Queue()
        for i in range(slots):
            self.free.put(i)
        self.jobs: "queue.Queue" = queue.Queue()
        self.errors: List[BaseException] = []
        self.written: List[str] = []
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def submit(self, wav: torch.Tensor, paths: Sequence[str]) -> None:
        """wav fp32 [B, C, N] on the device (postprocessed in place, as the reference's returned
        tensor); one WAV file per song."""
        B, C, N = wav.shape
        assert C == self.C and len(paths) == B
        for b in range(B):
            slot = self.free.get()
            if self.errors:
                raise RuntimeError("AudioWriter: a file write failed") from self.errors[0]
            n = N * C
            assert n <= self.pcm[slot].numel(), "AudioWriter: song longer than max_frames"
            pcm = self.pcm[slot][:n].view(1, N, C)
            postprocess_pcm16_(wav[b:b + 1], self.db, pcm)
            done = torch.cuda.Event()
            ready = torch.cuda.current_stream(self.device).record_event()
            self.copy_stream.wait_event(ready)
            with torch.cuda.stream(self.copy_stream):
                self.host[slot][:n].copy_(self.pcm[slot][:n], non_blocking=True)
                done.record(self.copy_stream)
            self.jobs.put((slot, n, done, paths[b]))

    def _run(self):
        while True:
            job = self.jobs.get()
            if job is None:
                return
            slot, n, done, path = job
            try:
                done.synchronize()
                write_wav_pcm16(path, self.host[slot][:n].view(-1, self.C), self.sr, self.C)
                self.written.append(path)
            except BaseException as e:  # surfaced on the next submit / flush
                self.errors.append(e)
            finally:
                self.free.put(slot)
                self.jobs.task_done()

    def flush(self) -> List[str]:
        self.jobs.join()
        if self.errors:
            raise RuntimeError("AudioWriter: a file write failed") from self.errors[0]
        out, self.written = self.written, []
        return out

    def close(self):
        self.flush()
        self.jobs.put(None)
        self._t.join()


def reference_host_leg(wav_dev: torch.Tensor, path: str, normalization_db: float = -1.0,
                       sample_rate: int = 48000) -> dict:
    """The reference's host leg for one song, timed step by step (bench.py's comparison): D→H of
    the fp32 audio (``pred_wavs[i].cpu()``), ``normalize_audio`` on the host tensor, the sample
    conversion soundfile applies before encoding (to [samples, channels] PCM16 frames), and the
    WAV write.  Returns per-step milliseconds and the frames written."""
    import time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a = wav_dev.cpu()                                          # generate_music_payload.py:41
    t1 = time.perf_counter()
    peak = torch.max(torch.abs(a))                             # audio_utils.py:36-57
    if not peak < 1e-6:
        a = a.clone() * (10 ** (normalization_db / 20.0) / peak)
    t2 = time.perf_counter()
    at = a.cpu().float().contiguous()                          # audio_utils.py:140-148
    frames = torch.round(torch.clamp(at.t(), -1.0, 1.0) * 32767.0).to(torch.int16).contiguous()
    t3 = time.perf_counter()
    write_wav_pcm16(path, frames, sample_rate, frames.shape[1])
    t4 = time.perf_counter()
    return {"d2h_ms": 1e3 * (t1 - t0), "normalize_ms": 1e3 * (t2 - t1), "convert_ms": 1e3 * (t3 - t2),
            "write_ms": 1e3 * (t4 - t3), "total_ms": 1e3 * (t4 - t0), "frames": frames}


def remove_quietly(paths: Sequence[str]) -> None:
    for p in paths:
        try:
            os.remove(p)
        except OSError:
            pass
