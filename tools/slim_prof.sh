#!/bin/bash
# Keep what a profile run is judged by (the rocprofv3 --stats summaries,
# the logs, prof_json.py's summary) and drop the raw per-dispatch databases,
# which exceed what gpurun copies back (64 MiB).  Usage: slim_prof.sh DIR
D=$1
for pass in trace fetch write sq; do
  [ -d "$D/$pass" ] || continue
  find "$D/$pass" -type f ! -name '*stats*' -delete
  find "$D/$pass" -type f -name '*stats*' -size +256k -exec gzip -9 {} +
done
exit 0
