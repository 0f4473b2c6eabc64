set -e
timeout -k 10 500 bash scripts/dev/p2m_pmc.sh
