"""Step processors (new/init/stats/norm/varsel/train/posttrain/eval/export/...)."""
