"""Per-frame path through the reference's own API: oracle/_ref/drop_in_enc
(the reference's hl_codec_encode with the gfx950 plugin installed, one frame
per call, host planes in and the slice NAL out) on the bench stream, with
the wall time of every hl_codec_encode call and every frame's output checked
against the reference encoder's MD5s (tests/golden/bench_golden.json).

  python tools/per_frame_api.py [frames] [name] [lookahead]     (name: bench_1088p_s11 or c2_720p_s7)

lookahead k > 1 runs the plugin's opt-in look-ahead (HL_AMD_LOOKAHEAD=k:
each hl_codec_encode returns the frame k - 1 calls earlier, the harness
drains the rest with hl_codec_264_gfx950_flush); all_fps = frames / (every
call's time + the flush), the first call (engine and buffer set-up) included.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hartallo_amd import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    name = sys.argv[2] if len(sys.argv) > 2 else "bench_1088p_s11"
    la = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_golden.json")))[name]
    w, h = g["width"], g["height"]
    clip = synth.clip(w, h, g["frames"], g["seed"])[:n]
    exe = os.path.join(ROOT, "oracle", "_ref", "drop_in_enc")
    with tempfile.TemporaryDirectory() as td:
        inp, out = os.path.join(td, "in.yuv"), os.path.join(td, "o.264")
        clip.tofile(inp)
        r = subprocess.run([exe, str(w), str(h), str(n), str(g["qp"]), str(g["me_range"]), str(g["deblock"]), str(g["gop"]), "0", inp, out],
                           capture_output=True, text=True, check=True, env=dict(os.environ, HL_AMD_LOOKAHEAD=str(la)))
        info = json.loads(r.stdout.strip().splitlines()[-1])
        stream = open(out, "rb").read()
    # per-frame check: the golden holds per-frame MD5s of the harness output
    pos, frames_ok = 0, True
    for i, (md5, nb) in enumerate(zip(g["frame_md5"][:n], g["frame_bytes"][:n])):
        frames_ok = frames_ok and hashlib.md5(stream[pos:pos + nb]).hexdigest() == md5
        pos += nb
    ms = info["encode_ms"]
    p_all = [m for i, m in enumerate(ms) if i % g["gop"]]  # every P picture
    p_warm = p_all[1:]  # without the first P picture (its call also allocates the run buffers)
    if la > 1:  # per-call times are those of queueing calls and of the calls that code a batch
        tot = sum(ms) + info.get("flush_ms", 0.0)
        print(json.dumps({"name": name, "width": w, "height": h, "frames": n, "lookahead": la, "bitexact": frames_ok and pos == len(stream),
                          "encode_ms": ms, "flush_ms": info.get("flush_ms"), "all_ms": round(tot, 2), "all_fps": round(1e3 * n / tot, 3),
                          "path": "hl_codec_encode (reference API) -> gfx950 plugin with HL_AMD_LOOKAHEAD -> hl_amd_encode's look-ahead "
                                  "(hl_amd_encode_batch per lookahead frames), then hl_codec_264_gfx950_flush"}), flush=True)
        return
    print(json.dumps({"name": name, "width": w, "height": h, "frames": n, "bitexact": frames_ok and pos == len(stream),
                      "encode_ms": ms,
                      "mean_p_ms": round(sum(p_all) / max(1, len(p_all)), 2),
                      "mean_p_ms_rule": "mean over every P picture of the call sequence, the first one included",
                      "mean_p_ms_after_first": round(sum(p_warm) / max(1, len(p_warm)), 2),
                      "p_fps": round(1e3 * len(p_all) / max(1e-9, sum(p_all)), 3),
                      "all_fps": round(1e3 * n / (sum(ms) + info.get("flush_ms", 0.0)), 3),
                      "path": "hl_codec_encode (reference API) -> gfx950 plugin -> hl_amd_encode, one frame per call"}), flush=True)


if __name__ == "__main__":
    main()
