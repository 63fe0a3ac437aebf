for lib in libzbot.so libzbot_nostage.so; do echo $lib; ZBOT_LIB=$lib timeout -k 10 120 python scripts/dev/diag_mgr.py 2>&1 | grep -v amdgpu.ids || exit 1; done
