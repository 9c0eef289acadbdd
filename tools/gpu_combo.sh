bash tools/gpu_ab3.sh $1 shockwave-replication_amd/lib/base.so && bash tools/gpu_c4prof.sh $1
