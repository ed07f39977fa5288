"""GPU child process of test_beam_small_grid_per_row_cross_tasks: one beam
search through the library named by WMI_LIB (a second build of the product
cannot share the test process's loaded library), with every step's logits
kept (WMI_LOGITS_ALL).  Writes tokens, score, the beam selections, the step
logits and the persistent grids used to an .npz file.

  WMI_LIB=... python tests/beam_worker.py MODEL_PATH SEED K N_TOK OUT.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "whisper.rs_amd")]
os.environ["WMI_LOGITS_ALL"] = "1"
import synth  # noqa: E402
import wmi  # noqa: E402


def main():
    path, seed, K, n_tok, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    ctx = wmi.WhisperContext.new(path, 0, max_clips=1)
    try:
        ctx.pcm_to_mel_batch([synth.synth_pcm_f32(30.0, seed)])
        ctx.encode(1, 0)
        toks, score = ctx.decode_beam(K, n_tok, suppress_eot=True)[0]
        np_ = 4 if ctx.special["multilingual"] else 2
        par, tok = ctx.beam_history(n_tok)
        np.savez(out, tokens=toks, score=np.float64(score), par=par, tok=tok,
                 logits=ctx.step_logits(np_ + n_tok - 1)[np_ - 1:, :K],
                 grids=np.frombuffer(ctx.debug_read(17, 9 * 4), np.int32).copy())
    finally:
        ctx.close()
    print(f"beam_worker: {wmi.LIB_PATH}: {len(toks)} tokens, score {score:.6f}")


if __name__ == "__main__":
    main()
