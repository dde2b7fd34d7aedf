bash tools/gpu_quick.sh r03h > gpurun_out/quick_r03h.txt 2>&1; rc=$?; cat gpurun_out/quick_r03h.txt | tail -12; [ $rc -eq 0 ] || exit $rc
bash tools/box_ab.sh "main fast fast2 main fast fast2" && bash tools/bvh_ab.sh "main fast main fast"
