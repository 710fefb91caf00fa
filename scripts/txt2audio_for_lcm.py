#!/usr/bin/env python3
"""Config-1 CLI (reference: scripts/txt2audio_for_lcm.py) on the MI355X path; see audiolcm_amd/cli.py.

  python scripts/txt2audio_for_lcm.py --prompt_txt prompts.txt --outdir out --ddim_steps 2 --sample_rate 16000 \
      -b configs/audiolcm.yaml -r model/000184.ckpt --vocoder-ckpt model/vocoder_bigvgan
  python scripts/txt2audio_for_lcm.py --test-dataset audiocaps --synthetic-seed 0 --ddim_steps 2 --outdir out
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from audiolcm_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    main(sys.argv[1:])
