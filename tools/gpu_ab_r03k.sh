#!/usr/bin/env bash
# same-box A/B (round 3, fast mode): box variants, then BVH (C5) variants, twice each
bash tools/box_ab.sh "base nskip base nskip" && bash tools/bvh_ab.sh "base lsel lroot both lf3 lf5 base lsel lroot both lf3 lf5"
