DataLoader = None  # trainer import only
