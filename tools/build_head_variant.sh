# Build the kernels + host ABI of a git revision as an A/B variant:
#   bash tools/build_head_variant.sh REV NAME  ->  gopacket_amd/build/libgpk_NAME.so
set -e
REV=${1:-HEAD}; NAME=${2:-head}
T=$(mktemp -d /tmp/gpk_rev.XXXXXX)
git archive "$REV" gopacket_amd/csrc include | tar -x -C "$T"
make -s -C "$T/gopacket_amd/csrc" variant V="$NAME" > /dev/null
mkdir -p gopacket_amd/build
cp "$T/gopacket_amd/build/libgpk_$NAME.so" gopacket_amd/build/
rm -rf "$T"
