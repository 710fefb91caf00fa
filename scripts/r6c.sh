#!/bin/bash
bash scripts/diag_tail.sh r6c_diag && bash scripts/pmc_w3.sh r6c_w3
