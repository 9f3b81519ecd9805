"""MI355X-native region-proposal + RoI hot path of replication_faster_rcnn."""
