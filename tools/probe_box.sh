set -x
nproc; lscpu | head -20; ldconfig -p | grep -i sodium; ls -la /opt/conda/lib/libsodium* ; 
rocminfo | grep -E "Marketing|Compute Unit|Max Clock|gfx" | head -20
timeout -k 10 120 ./tools/ubench_valu
