set -e
mkdir -p gpurun_out
for lib in text_guided_face_recognition_amd/lib/libtgfr_hip.so text_guided_face_recognition_amd/lib/var/libtgfr_nostore.so text_guided_face_recognition_amd/lib/var/libtgfr_NOMFMA.so text_guided_face_recognition_amd/lib/var/libtgfr_NOLOAD.so; do
  for cfg in 1; do
    echo -n "$(basename $lib) cfg$cfg: "
    TGFR_LIB=$lib TGFR_GEMM_CFG=$cfg timeout -k 10 60 python tools/gemm_exp.py
  done
done
