#!/usr/bin/env bash
# same-box A/B (round 3, fast mode): tunables re-swept after the arithmetic-mode change
bash tools/bvh_ab.sh "base rf5 rf7 ll4 st2 leaf4 leaf8 base rf5 rf7 ll4 st2 leaf4 leaf8" && bash tools/box_ab.sh "base rb32 rb48 dg0 base rb32 rb48 dg0" && bash tools/box_ab.sh "base rb32 rb48 dg0" box_mirror
