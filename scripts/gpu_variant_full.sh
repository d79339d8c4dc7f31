# A prebuilt variant (var_libs/$V) in place of the library: parity tests, exec diag, bench.
set -e
R=$GRAFT_REPO_ROOT
cp $R/var_libs/$V/libdeltareplay.so $R/delta_amd/libdeltareplay.so
bash $R/scripts/gpu_exec_iter.sh
