set -u
timeout -k 10 60 ./tools/capacity_probe || exit 1
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_var_tenv.so mlx-data_amd/libmxd_amd.so
timeout -k 10 200 python tools/band_sweep.py --workload c4 --reps 5 --set wrows=0 --set wrows=8 --set wrows=12 --set wrows=14 --set wrows=16 --set wrows=19 --set wrows=23
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
