"""Data ingestion with the reference's module layout (`from data.video_dataset import ...`)."""
