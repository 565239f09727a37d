export LIBS="libslam_hip.so libslam_norng.so libslam_noepi.so libslam_noslow.so libslam_nolik.so libslam_wpe0.so"
TAG=var3a tools/variants_run.sh && tools/pmc_variants.sh
