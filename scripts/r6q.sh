#!/bin/bash
# round 6, call q: wconv3 persistent grid on a part of the chip for the BigVGAN stage 0-2 convs (ALCM_XP0 = workgroups)
# so the three resblock chains' convs run side by side, headline alternating
TESTS=0 ROUNDS=2 bash scripts/gpu_ab.sh r6q_ab "ALCM_XP0=0" "ALCM_XP0=88" "ALCM_XP0=128" "ALCM_XP0=176"
